// Shared device helpers for the gfx950 (CDNA4) kernels of liblci.
// Wave = 64 lanes. MFMA fragments follow the gfx950 lane maps (cdna_hip_programming.md §3):
//   v_mfma_f32_32x32x16_bf16: lane l (r = l&31, h = l>>5) holds A[r][8h+j], B[8h+j][r], j=0..7;
//   C/D reg i of lane l is C[(i&3) + 8*(i>>2) + 4*h][l&31].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lci {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define LCI_LDS __attribute__((address_space(3)))

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

// f32 -> bf16 round-to-nearest-even (hipcc lowers the cast to v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ bf16 to_bf16(float x) { return (bf16)x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }

// Pack 8 consecutive accumulator registers (8s..8s+7) into a bf16x8 operand fragment.
template <int S>
__device__ __forceinline__ bf16x8 pack8(const f32x16& c) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = to_bf16(c[8 * S + j]);
  return r;
}

// Transposed LDS read (ds_read_b64_tr_b16): per 16-lane group a 4-row x 16-col bf16 block.
__device__ __forceinline__ bf16x4 lds_tr4(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((LCI_LDS bf16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat44(bf16x4 a, bf16x4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// A-operand fragment of X^T for an LDS tile X[row][col] (bf16, row stride `ld` elements), where the MFMA
// sums over X's ROW index in the permuted k-order of an accumulator used as the other operand
// (element j of half h <-> row r0 + 16s + 8(j>>2) + 4h + (j&3)), and the MFMA row is X's column c0 + (l&31).
template <int S>
__device__ __forceinline__ bf16x8 frag_tr(const bf16* tile, int ld, int r0, int c0, int lane) {
  const int row = r0 + 16 * S + 4 * (lane >> 5) + ((lane & 15) >> 2);
  const int col = c0 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  bf16x4 lo = lds_tr4(tile + row * ld + col);
  bf16x4 hi = lds_tr4(tile + (row + 8) * ld + col);
  return cat44(lo, hi);
}

// Row fragment (A of rows r0+(l&31), or B^T of cols): 8 consecutive bf16 of row r0+(l&31) at col c0+8h.
__device__ __forceinline__ bf16x8 frag_row(const bf16* tile, int ld, int r0, int c0, int lane) {
  return *(const bf16x8*)(tile + (r0 + (lane & 31)) * ld + c0 + 8 * (lane >> 5));
}

// Buffer resource over `bytes` bytes from `base` (raw, range-checked: a load whose offset + size exceeds `bytes`
// returns zeros) and a 16-byte load through it (per-lane 32-bit offset + wave-uniform offset).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload16(rsrc_t r, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
}

// LDS-DMA of one 1-KB unit (buffer_load_dwordx4 ... lds): lane l's 16 bytes at (voff + soff) of resource r land at
// LDS byte lds + 16 l (m0 holds the wave-uniform LDS base; saved and restored around the load). Range-checked like
// bload16: out-of-range lanes write zeros.
__device__ __forceinline__ void dma16_lds(rsrc_t r, int voff, int soff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds), "s"(soff) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {   // s_waitcnt vmcnt(N), lgkmcnt / expcnt untouched (gfx9 encoding)
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  __builtin_amdgcn_sched_barrier(0);
}

// Combine lane l with lane l^32 (the two halves of a 32x32 MFMA column): one v_permlane32_swap, no LDS.
__device__ __forceinline__ float wave_max_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_sum_xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

}  // namespace lci

// ------------------------------------------------------------------ host-side error plumbing
namespace lci {
void set_error(const char* fmt, ...);
}

#define LCI_CHECK(cond, ...)           \
  do {                                 \
    if (!(cond)) {                     \
      lci::set_error(__VA_ARGS__);     \
      return 1;                        \
    }                                  \
  } while (0)

#define LCI_HIP(call)                                                             \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      lci::set_error("%s failed: %s", #call, hipGetErrorString(e_));              \
      return 2;                                                                   \
    }                                                                             \
  } while (0)

#define LCI_LAUNCH_CHECK()                                                        \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      lci::set_error("kernel launch failed: %s", hipGetErrorString(e_));          \
      return 3;                                                                   \
    }                                                                             \
  } while (0)
