// Shared device/host helpers for the MI355X (gfx950) NeRF kernels.
// Conventions of the C-ABI (include/nerf_amd.h): raw device pointers, explicit
// hipStream_t, int status (0 ok, <0 error), thread-local nerf_last_error(), no allocation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#ifndef NERF_HOST_ONLY
namespace nerf {

constexpr int WAVE = 64;

// ------------------------------------------------------------------------------------
// error plumbing (host)
// ------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int check_launch(const char* what);  // reads hipGetLastError(), maps to status

#define NERF_REQUIRE(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::nerf::set_error(__VA_ARGS__);      \
      return -22; /* EINVAL */             \
    }                                      \
  } while (0)

// ------------------------------------------------------------------------------------
// IEEE single ops that must not be contracted into FMA (torch CPU evaluates them as
// separately rounded ops; bit-parity of sampling/indices depends on it).
// ------------------------------------------------------------------------------------
// hipcc contracts a*b+c into v_fma_f32 by default (-ffp-contract=fast) even through
// __fmul_rn/__fadd_rn; the pragma keeps the `contract` flag off these instructions so
// they stay separately rounded after inlining.
__device__ __forceinline__ float fmul(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float fadd(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float fsub(float a, float b) {
#pragma clang fp contract(off)
  return a - b;
}
__device__ __forceinline__ float fdiv(float a, float b) {
#pragma clang fp contract(off)
  return a / b;  // IEEE division (hipcc default: correctly rounded f32 div)
}

// ------------------------------------------------------------------------------------
// counter-based RNG: a Philox-4x32-10 stream keyed by (seed) and counted by (offset, idx)
// -> uniform float in [0,1) with 24 random bits.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c.x, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c.z, &hi1);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float rng_uniform(uint64_t seed, uint64_t offset, uint64_t idx) {
  uint4 c = make_uint4((uint32_t)idx, (uint32_t)(idx >> 32), (uint32_t)offset, (uint32_t)(offset >> 32));
  uint4 r = philox(c, make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  return u01(r.x);
}

// ------------------------------------------------------------------------------------
// wave helpers (64 lanes)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ float shfl(float v, int src) { return __shfl(v, src, 64); }
__device__ __forceinline__ double shfl_d(double v, int src) { return __shfl(v, src, 64); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// torch.sum(x, -1) of one contiguous fp32 row on the CPU, bit for bit, for n <= 64 values held
// one per lane (x_i on lane i, any value beyond n).  sample_pdf normalises by this sum
// (volume_renderer.py:91-92) and a trained net's fine samples move by an ulp with it (an
// 800x800 silhouette pixel: 3.4e-5 of rgb per ulp), so the order is ATen's, not a tree:
// vectorized_inner_sum (SumKernel.cpp) over 8-lane float vectors v_j = x[8j, 8j+8), j < nv =
// n/8: row_sum's ilp-4 partials p_k = sum_r v_{4r+k} (r < nv/4, multi_row_sum below its first
// 16-row level), the leftover vectors added to p_0, then p_0 + p_1 + p_2 + p_3; the scalar tail
// x[8nv, n) summed from 0, then the 8 vector lanes added in order.  Matches torch 2.10 CPU on
// every one of 20,000 random 62-value rows (tree sum: 52 %, fp64: 57 %).  The order is that of
// torch CPU with 8-float vectors: on the x86 host the goldens were made on (AVX512-capable),
// ATEN_CPU_CAPABILITY=avx512 / avx2 / default give the same sums bit for bit (sum_stub runs
// on 32-byte vectors in all three); a build with 16-float sum vectors, or the reference run
// on CUDA (another reduction order), is not what this pins.
__device__ __forceinline__ float torch_row_sum(float x, int n) {
  const int j = lane_id() & 7;
  const int nv = n >> 3, nilp = nv >> 2;
  float p[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    p[k] = 0.f;
    for (int r = 0; r < nilp; ++r) p[k] = fadd(p[k], __shfl(x, (4 * r + k) * 8 + j, 64));
  }
  for (int i = 4 * nilp; i < nv; ++i) p[0] = fadd(p[0], __shfl(x, 8 * i + j, 64));
  const float p0 = fadd(fadd(fadd(p[0], p[1]), p[2]), p[3]);
  float s = 0.f;
  for (int k = 8 * nv; k < n; ++k) s = fadd(s, __shfl(x, k, 64));
#pragma unroll
  for (int k = 0; k < 8; ++k) s = fadd(s, __shfl(p0, k, 64));
  return s;
}

// inclusive product scan across the wave, in double (torch CPU cumprod accumulates in
// double; the exact sum/product of <=256 fp32 terms rarely needs more than 53 bits).
__device__ __forceinline__ double wave_scan_mul(double v) {
  int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double t = __shfl_up(v, o, 64);
    if (l >= o) v *= t;
  }
  return v;
}
__device__ __forceinline__ double wave_scan_add(double v) {
  int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    double t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}
__device__ __forceinline__ float wave_scan_add_f(float v) {
  int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    float t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

}  // namespace nerf
#endif
