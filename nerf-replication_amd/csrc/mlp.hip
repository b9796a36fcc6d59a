// Fused NeRF MLP on gfx950 MFMA: positional encoding + 8x256 trunk (skip@4) + alpha /
// feature / view branch, forward and backward.
//
// Replaces the ATen op sequence of Network.forward / NeRF.forward
// (src/models/nerf/network.py:49-74, 171-192; encoders src/models/encoding/freq.py:7-32)
// and its autograd backward.
//
// Kernels:
//   pack_kernel   fp32 nn.Linear weights -> lane-linear A-operand chunks (W for the
//                 forward, W^T for the dX chain) + per-unit bias chunks
//   fwd_kernel    one wave = 32 samples through all 11 layers; activations never leave
//                 registers; weights stream through a 2-slot LDS ring filled by
//                 global_load_lds, one unit (one 32-row output tile of one layer) per slot.
//                 The training variant also stores every layer input feature-major and
//                 the ReLU masks.
//   dx_kernel     the dX chain (W^T products + ReLU masks), 32 samples per wave, storing
//                 every layer's output gradient feature-major
//   dw_kernel     dW/db = dz . act^T, a K = samples GEMM per layer; fp32 atomics combine
//                 sample chunks
#include "common.h"
#include "mlp_tables.h"

#include <mutex>
#include <type_traits>
#include <utility>

namespace nerf {
namespace mlp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// mask bits of the bf16x3 training forward from the packed hi pair (v_pk_min_u16 + v_lshl_or_b32
// per register pair) instead of per-value compares and selects
#ifndef NERF_PACKED_MASK
#define NERF_PACKED_MASK 1
#endif

// registers 2k, 2k+1 of an fp32 accumulator as one packed bf16 pair (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, bf16x2));
}

// ------------------------------------------------------------------------------------
// precision policies
// ------------------------------------------------------------------------------------
enum PKind { K_F32 = 0, K_BF16 = 1, K_BF16X3 = 2, K_BF16X6 = 3, K_BF16X3W = 4, K_F32W = 5, K_BF16W = 6 };

struct PF32 {
  static constexpr int KIND = K_F32;
  using Acc = f32x16;     // one 32x32 accumulator tile
  static constexpr int SPW = 32;  // samples per wave
  static constexpr int CH = 4;     // 1 KiB chunks per 32-feature input tile
  static constexpr int E = 4;      // elements per lane per chunk
  static constexpr int WAVES = 4;  // one wave per SIMD (<= 512 VGPR+AGPR)
  static constexpr int ESIZE = 4;
  static constexpr int SPL = 4;    // samples per 16-B lane load (dW GEMM)
  static constexpr int PE = 1;  // PE_LIBM: the fp32 parity path (pe_trig)
  using Store = float;
  struct Tile { float v[16]; };
  static __device__ __forceinline__ f32x16 mma(uint4 a, const Tile& b, int c, f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), b.v[4 * c + 0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), b.v[4 * c + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), b.v[4 * c + 2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), b.v[4 * c + 3], acc, 0, 0, 0);
    return acc;
  }
  static __device__ __forceinline__ void set(Tile& t, int rho, float x) { t.v[rho] = x; }
  // a whole tile from its 16 register values
  static __device__ __forceinline__ void pack16(Tile& t, const float (&v)[16]) {
#pragma unroll
    for (int rho = 0; rho < 16; ++rho) t.v[rho] = v[rho];
  }
  static __device__ __forceinline__ float get(const Tile& t, int rho) { return t.v[rho]; }
  static __device__ __forceinline__ Store cvt(float x) { return x; }
  // packed weight element e of chunk c: accumulator register (k order) and stored value
  static __host__ __device__ constexpr int rho_of(int c, int e) { return c * E + e; }
  static __device__ __forceinline__ Store cvt_c(float x, int) { return x; }
  static __device__ __forceinline__ f32x16 mma_k(uint4 a, uint4 b, f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
    return acc;
  }
  static __device__ __forceinline__ float lsum(uint4 a) {
    return ((__uint_as_float(a.x) + __uint_as_float(a.y)) + __uint_as_float(a.z)) + __uint_as_float(a.w);
  }
  static __device__ __forceinline__ uint4 chunk(const Tile& t, int c) {
    return make_uint4(__float_as_uint(t.v[4 * c]), __float_as_uint(t.v[4 * c + 1]), __float_as_uint(t.v[4 * c + 2]),
                      __float_as_uint(t.v[4 * c + 3]));
  }
  // registers 2k, 2k + 1 of a tile (the finish writes a tile pair by pair)
  static __device__ __forceinline__ void set_pair(Tile& t, int k, float x0, float x1) {
    t.v[2 * k] = x0;
    t.v[2 * k + 1] = x1;
  }
};

struct PBF16 {
  static constexpr int KIND = K_BF16;
  using Acc = f32x16;     // one 32x32 accumulator tile
  static constexpr int SPW = 32;  // samples per wave
  static constexpr int CH = 2;
  static constexpr int E = 8;
  static constexpr int WAVES = 8;  // two waves per SIMD (<= 256 VGPR)
  static constexpr int ESIZE = 2;
  static constexpr int SPL = 8;
  static constexpr int PE = 0;  // PE_FAST: rounded to bf16 anyway
  using Store = __bf16;
  struct Tile { bf16x8 b[2]; };
  static __device__ __forceinline__ f32x16 mma(uint4 a, const Tile& b, int c, f32x16 acc) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), b.b[c], acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void set(Tile& t, int rho, float x) { t.b[rho >> 3][rho & 7] = (__bf16)x; }
  static __device__ __forceinline__ void pack16(Tile& t, const float (&v)[16]) {
    uint32_t d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
    t.b[0] = __builtin_bit_cast(bf16x8, make_uint4(d[0], d[1], d[2], d[3]));
    t.b[1] = __builtin_bit_cast(bf16x8, make_uint4(d[4], d[5], d[6], d[7]));
  }
  static __device__ __forceinline__ float get(const Tile& t, int rho) { return (float)t.b[rho >> 3][rho & 7]; }
  static __device__ __forceinline__ Store cvt(float x) { return (__bf16)x; }
  static __host__ __device__ constexpr int rho_of(int c, int e) { return c * E + e; }
  static __device__ __forceinline__ Store cvt_c(float x, int) { return (__bf16)x; }
  static __device__ __forceinline__ f32x16 mma_k(uint4 a, uint4 b, f32x16 acc) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
  static __device__ __forceinline__ float lsum(uint4 a) {
    bf16x8 v = __builtin_bit_cast(bf16x8, a);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += (float)v[i];
    return s;
  }
  static __device__ __forceinline__ uint4 chunk(const Tile& t, int c) { return __builtin_bit_cast(uint4, t.b[c]); }
  // packed pair k (registers 2k, 2k + 1) = dword k & 3 of chunk k >> 2
  static __device__ __forceinline__ void set_dword(Tile& t, int k, uint32_t d) {
    uint4 v = __builtin_bit_cast(uint4, t.b[k >> 2]);
    if ((k & 3) == 0) v.x = d;
    else if ((k & 3) == 1) v.y = d;
    else if ((k & 3) == 2) v.z = d;
    else v.w = d;
    t.b[k >> 2] = __builtin_bit_cast(bf16x8, v);
  }
  static __device__ __forceinline__ void set_pair(Tile& t, int k, float x0, float x1) {
    set_dword(t, k, pack_bf16(x0, x1));
  }
};

// bf16x3: every fp32 operand x is split x = hi + lo (hi = bf16(x), lo = bf16(x - hi), 16
// significant bits together) and a product is hi*hi + hi*lo + lo*hi on the bf16 MFMA with fp32
// accumulation -- 3 bf16 MFMAs (96 cycles) per K = 16 step instead of 8 fp32 ones (512 cycles),
// at ~1e-5 relative error per dot product (fp32-class; the fp32 parity tests hold at 1e-4).
// Weights: chunks 0, 1 = hi of k 0-7 / 8-15, chunks 2, 3 = lo.  Tiles hold hi and lo (16
// VGPRs, as fp32), stored as 4 KiB tile-blocks (hi 2 KiB then lo 2 KiB).
struct PBF3 {
  static constexpr int KIND = K_BF16X3;
  using Acc = f32x16;     // one 32x32 accumulator tile
  static constexpr int SPW = 32;  // samples per wave
  static constexpr int CH = 4;
  static constexpr int E = 8;
  static constexpr int WAVES = 4;  // one wave per SIMD (16-VGPR tiles)
  static constexpr int ESIZE = 4;
  static constexpr int SPL = 8;
  static constexpr int PE = 2;  // PE_POLY: fp32-accurate to 1.6 ulp, then split
  using Store = __bf16;
  struct Tile { bf16x8 hi[2], lo[2]; };
  static __device__ __forceinline__ f32x16 mma(uint4 a, const Tile& b, int c, f32x16 acc) {
    const bf16x8 av = __builtin_bit_cast(bf16x8, a);
    if (c < 2) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, b.hi[c], acc, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, b.lo[c], acc, 0, 0, 0);
    }
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, b.hi[c - 2], acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void set(Tile& t, int rho, float x) {
    const __bf16 h = (__bf16)x;
    t.hi[rho >> 3][rho & 7] = h;
    t.lo[rho >> 3][rho & 7] = (__bf16)(x - (float)h);
  }
  // packed pairs: hi = v_cvt_pk_bf16_f32, its fp32 value by a shift / mask, lo = the
  // residuals' pair (same values as set(), 4 VALU per pair instead of element inserts)
  static __device__ __forceinline__ void pack16(Tile& t, const float (&v)[16]) {
    uint32_t hw[8], lw[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      hw[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
      lw[k] = pack_bf16(v[2 * k] - __uint_as_float(hw[k] << 16), v[2 * k + 1] - __uint_as_float(hw[k] & 0xffff0000u));
    }
    t.hi[0] = __builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
    t.hi[1] = __builtin_bit_cast(bf16x8, make_uint4(hw[4], hw[5], hw[6], hw[7]));
    t.lo[0] = __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
    t.lo[1] = __builtin_bit_cast(bf16x8, make_uint4(lw[4], lw[5], lw[6], lw[7]));
  }
  static __device__ __forceinline__ float get(const Tile& t, int rho) {
    return (float)t.hi[rho >> 3][rho & 7] + (float)t.lo[rho >> 3][rho & 7];
  }
  static __host__ __device__ constexpr int rho_of(int c, int e) { return (c & 1) * E + e; }
  static __device__ __forceinline__ Store cvt_c(float x, int c) {
    const __bf16 h = (__bf16)x;
    return c < 2 ? h : (__bf16)(x - (float)h);
  }
  static __device__ __forceinline__ uint4 chunk(const Tile& t, int c) {
    return __builtin_bit_cast(uint4, c < 2 ? t.hi[c] : t.lo[c - 2]);
  }
  static __device__ __forceinline__ void put(bf16x8& dst, int q, uint32_t d) {
    uint4 v = __builtin_bit_cast(uint4, dst);
    if (q == 0) v.x = d;
    else if (q == 1) v.y = d;
    else if (q == 2) v.z = d;
    else v.w = d;
    dst = __builtin_bit_cast(bf16x8, v);
  }
  // registers 2k, 2k + 1 split into hi / lo pairs (the values pack16 gives)
  static __device__ __forceinline__ void set_pair(Tile& t, int k, float x0, float x1) {
    const uint32_t hw = pack_bf16(x0, x1);
    const uint32_t lw = pack_bf16(x0 - __uint_as_float(hw << 16), x1 - __uint_as_float(hw & 0xffff0000u));
    put(t.hi[k >> 2], k & 3, hw);
    put(t.lo[k >> 2], k & 3, lw);
  }

};

// bf16x6 (inference forward only, round 5): every fp32 operand split exactly into three bf16,
// x = hi + mid + lo (24 significant bits), and the six products hh, hm, mh, hl, lh, mm accumulated in
// fp32 on the bf16 MFMA (the dropped ml, lm, ll are < 2^-24 relative): at least as accurate as an fp32
// GEMM, at 6 bf16 MFMAs (192 cycles) per K = 16 step instead of 8 fp32 ones (512).  The render of the
// bf16x3 tiers evaluates its COARSE net with it (Network.mlp_dtype_for): a split-bf16 coarse net moves
// importance samples across CDF bins.  Activations stay fp32 in registers (16
// VGPRs per tile, as PF32) and are split when a K half is used (12 VGPRs live at a time): the chunk
// order hi, mid, lo of K half 0, then of K half 1, so the split of one half is reused by its three
// chunks.  Weights: chunk 3q + p = part p (hi / mid / lo) of K half q.
struct PBF6 {
  static constexpr int KIND = K_BF16X6;
  using Acc = f32x16;     // one 32x32 accumulator tile
  static constexpr int SPW = 32;  // samples per wave
  static constexpr int CH = 6;
  static constexpr int E = 8;
  static constexpr int WAVES = 4;  // one wave per SIMD (16-VGPR fp32 tiles)
  static constexpr int ESIZE = 4;
  static constexpr int SPL = 8;
  static constexpr int PE = 2;  // PE_POLY: fp32-accurate to 1.6 ulp
  using Store = __bf16;
  struct Tile { float v[16]; };
  struct Split { bf16x8 h, m, l; };
  // K half q (registers 8q .. 8q + 7) as three bf16x8 parts
  static __device__ __forceinline__ Split split(const Tile& t, int q) {
    uint32_t hw[4], mw[4], lw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x0 = t.v[8 * q + 2 * k], x1 = t.v[8 * q + 2 * k + 1];
      hw[k] = pack_bf16(x0, x1);
      const float r0 = x0 - __uint_as_float(hw[k] << 16), r1 = x1 - __uint_as_float(hw[k] & 0xffff0000u);
      mw[k] = pack_bf16(r0, r1);
      lw[k] = pack_bf16(r0 - __uint_as_float(mw[k] << 16), r1 - __uint_as_float(mw[k] & 0xffff0000u));
    }
    return Split{__builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3])),
                 __builtin_bit_cast(bf16x8, make_uint4(mw[0], mw[1], mw[2], mw[3])),
                 __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]))};
  }
  static __device__ __forceinline__ f32x16 mma(uint4 a, const Tile& b, int c, f32x16 acc) {
    const bf16x8 av = __builtin_bit_cast(bf16x8, a);
    const int q = c / 3, p = c % 3;
    const Split x = split(b, q);  // (identical for the three chunks of a half: CSE'd)
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, x.h, acc, 0, 0, 0);
    if (p == 2) return acc;                                                  // lo . hi
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, x.m, acc, 0, 0, 0);   // . mid
    if (p == 1) return acc;
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, x.l, acc, 0, 0, 0);  // hi . lo
  }
  static __device__ __forceinline__ void set(Tile& t, int rho, float x) { t.v[rho] = x; }
  static __device__ __forceinline__ void pack16(Tile& t, const float (&v)[16]) {
#pragma unroll
    for (int rho = 0; rho < 16; ++rho) t.v[rho] = v[rho];
  }
  static __device__ __forceinline__ float get(const Tile& t, int rho) { return t.v[rho]; }
  static __host__ __device__ constexpr int rho_of(int c, int e) { return (c / 3) * E + e; }
  static __device__ __forceinline__ Store cvt_c(float x, int c) {
    const __bf16 h = (__bf16)x;
    const float r = x - (float)h;
    const __bf16 m = (__bf16)r;
    return c % 3 == 0 ? h : c % 3 == 1 ? m : (__bf16)(r - (float)m);
  }
  static __device__ __forceinline__ void set_pair(Tile& t, int k, float x0, float x1) {
    t.v[2 * k] = x0;
    t.v[2 * k + 1] = x1;
  }
};

// bf16x3 on v_mfma_f32_16x16x32_bf16 (round 6, the "wide" bf16x3 forward: 16 samples per wave, 8
// waves per workgroup = two per SIMD, so that one wave's epilogue runs beside the other's MFMAs).  The
// same arithmetic as PBF3 -- every fp32 operand split x = hi + lo, products hi*hi + hi*lo + lo*hi with
// fp32 accumulation -- on 16-row units (mlp_tables.h fwd16_*).  A chunk is 16 weight rows x one 32-feature
// K-block: chunk 0 the hi halves, chunk 1 the lo halves; a Tile is one K-block of the B operand (8 hi +
// 8 lo bf16 per lane, 8 VGPRs), the accumulator 4 fp32.  Forward only: the bf16x3 dX / dW and the bf16
// backward of bf16x3f read its training stores, which it writes in the 32x32 fragment layout.
struct PBF3W {
  static constexpr int KIND = K_BF16X3W;
  using Acc = f32x4;
  static constexpr int SPW = 16;
  static constexpr int CH = 2;
  static constexpr int E = 8;
  static constexpr int WAVES = 8;
  static constexpr int ESIZE = 4;
  static constexpr int SPL = 8;
  static constexpr int PE = 2;  // PE_POLY, as PBF3
  using Store = __bf16;
  struct Tile { bf16x8 hi, lo; };
  static __device__ __forceinline__ f32x4 mma(uint4 a, const Tile& b, int c, f32x4 acc) {
    const bf16x8 av = __builtin_bit_cast(bf16x8, a);
    if (c == 0) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b.hi, acc, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b.lo, acc, 0, 0, 0);
    }
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, b.hi, acc, 0, 0, 0);
  }
  static __host__ __device__ constexpr int rho_of(int, int e) { return e; }  // (a chunk reads the whole K-block)
  static __device__ __forceinline__ Store cvt_c(float x, int c) {
    const __bf16 h = (__bf16)x;
    return c == 0 ? h : (__bf16)(x - (float)h);
  }
  // packed weight element e of chunk c, lane group g: feature k16_feat(g, e) of the K-block, split part c
  static __host__ __device__ constexpr int feat16(int, int g, int e) { return k16_feat(g, e); }
  static __host__ __device__ constexpr int part16(int c) { return c; }
};

// The wide fp32 TRAINING forward (round 6, PF32W): the PBF3W structure on v_mfma_f32_16x16x4_f32 -- one wave =
// 16 samples, 8 waves per workgroup, two per SIMD (the 32x32x2 fp32 forward holds 32 samples' fp32 tiles in
// ~450 registers: one wave per SIMD).  A K-block (32 features x 16 samples) is 8 MFMAs; MFMA j's B operand in
// lane (s, g) is feature 16 (j >> 2) + 4 g + (j & 3) = k16_feat(g, j), so a 16x16 output tile mt (rows 4 g + e
// in lane g) IS registers 4 (mt & 1) + e of the next layer's K-block mt >> 1.  Chunk c (1 KiB) of a K-block =
// MFMAs 4c .. 4c + 3: lane l = r16 + 16 g reads W[r16][16 c + 4 g + 0..3], four contiguous fp32.  Same
// arithmetic as PF32 (fp32 products, fp32 accumulation, libm PE), another summation order: the training forward
// only -- renders keep PF32's order, which the full-frame fixtures are pinned against.
struct PF32W {
  static constexpr int KIND = K_F32W;
  using Acc = f32x4;
  static constexpr int SPW = 16;
  static constexpr int CH = 2;
  static constexpr int E = 4;
  static constexpr int WAVES = 8;
  static constexpr int ESIZE = 4;
  static constexpr int SPL = 4;
  static constexpr int PE = 1;  // PE_LIBM, as PF32
  using Store = float;
  struct Tile { float v[8]; };
  static __device__ __forceinline__ f32x4 mma(uint4 a, const Tile& b, int c, f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), b.v[4 * c + 0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), b.v[4 * c + 1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), b.v[4 * c + 2], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), b.v[4 * c + 3], acc, 0, 0, 0);
  }
  static __host__ __device__ constexpr int rho_of(int c, int e) { return 4 * c + e; }
  static __device__ __forceinline__ Store cvt_c(float x, int) { return x; }
  static __host__ __device__ constexpr int feat16(int c, int g, int e) { return 16 * c + 4 * g + e; }
  static __host__ __device__ constexpr int part16(int) { return 0; }
};
// The wide bf16 dX (round 6, PBF16W): the bf16 dX of the bf16 and bf16x3f tiers on v_mfma_f32_16x16x32_bf16 over the
// 16-row W^T units -- PBF3W's layout with the hi half only (one 1 KiB chunk per K-block).
struct PBF16W {
  static constexpr int KIND = K_BF16W;
  using Acc = f32x4;
  static constexpr int SPW = 16;
  static constexpr int CH = 1;
  static constexpr int E = 8;
  static constexpr int WAVES = 8;
  static constexpr int ESIZE = 2;
  static constexpr int SPL = 8;
  static constexpr int PE = 0;
  using Store = __bf16;
  struct Tile { bf16x8 hi; };
  static __device__ __forceinline__ f32x4 mma(uint4 a, const Tile& b, int, f32x4 acc) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), b.hi, acc, 0, 0, 0);
  }
  static __host__ __device__ constexpr int rho_of(int, int e) { return e; }
  static __device__ __forceinline__ Store cvt_c(float x, int) { return (__bf16)x; }
  static __host__ __device__ constexpr int feat16(int, int g, int e) { return k16_feat(g, e); }
  static __host__ __device__ constexpr int part16(int) { return 0; }
};
template <class P> __host__ __device__ constexpr bool wide_kind() {
  return P::KIND == K_BF16X3W || P::KIND == K_F32W || P::KIND == K_BF16W;
}

// ReLU-mask bit of accumulator register rho of a tile: the tile's 16 bits sit at positions
// (rho >> 1) + 16 (rho & 1) of a dword (bf16 pair k = registers 2k, 2k+1 -> bits k, 16 + k),
// and two tiles n, n + 1 share one dword, the odd one shifted up by 8.
__host__ __device__ constexpr int mask_bit(int rho) { return (rho >> 1) + 16 * (rho & 1); }

typedef __attribute__((ext_vector_type(2))) short i16x2;
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
// ReLU of a bf16 pair: sign-magnitude bf16 ordered as int16 -> v_pk_max_i16 with 0
// (relu(bf16(x)) == bf16(relu(x)): rounding keeps the sign)
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t d) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(i16x2, d), (i16x2){0, 0}));
}
// 1 in each half that is non-zero: v_pk_min_u16 with `one` = 0x00010001, which the caller holds in an
// SGPR laundered through an empty asm (no instruction) -- hipcc then emits the one v_pk_min_u16 itself;
// knowing the operand is 1 it rewrites min(x, 1) into a compare and a select per half.
// Round 6: this WAS an inline-asm v_pk_min_u16.  hipcc's hazard recognizer does not model the MFMA
// hazards of an inline-asm VGPR write: with finish parts 2 it allocated the asm's output to v1, a dead
// lane of the rgb unit's accumulator v[0:15] whose MFMA had issued one instruction earlier and still
// had its write of v[0:15] pending -- the MFMA's late write-back replaced the mask bits on some runs
// (the round-5 "masks differ run to run" finding; tools/mfma_war_scan.py: asm write 1 wait state after
// the MFMA, against >= 13 for every compiler-placed write).  No VGPR-writing inline asm is left in the
// MFMA kernels (tools/asm_check.py fails one).
__device__ __forceinline__ uint32_t nonzero_bf16x2(uint32_t d, uint32_t one) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, d), __builtin_bit_cast(u16x2, one)));
}
__device__ __forceinline__ uint32_t opaque_one16() {
  uint32_t one = 0x00010001u;
  asm("" : "+s"(one));
  return one;
}

template <class P> __host__ __device__ constexpr int samples_per_block() { return P::WAVES * P::SPW; }
constexpr int M_ALIGN = 256;  // activation stores are padded to this many samples

// ------------------------------------------------------------------------------------
// packed-weight layout (1 KiB chunks, lane-linear: chunk[lane][16 B])
//   forward unit u: fwd_unit_tiles(u) * CH weight chunks, then 1 bias chunk (32 fp32)
//   backward unit u: bwd_unit_tiles(u) * CH weight chunks
// ------------------------------------------------------------------------------------
// DIR 0: forward units, 1: dX-chain units, 2: 16-row forward units (PBF3W)
// DIR 3: 16-row dX units (PF32W / PBF3W)
__host__ __device__ constexpr int num_units(int dir) {
  return dir == 0 ? NUNIT_FWD : dir == 1 ? NUNIT_BWD : dir == 2 ? NUNIT_FWD16 : NUNIT_BWD16;
}
__host__ __device__ constexpr int fwd_unit_chunks(int u, int ch) { return fwd_unit_tiles(u) * ch + 1; }
__host__ __device__ constexpr int fwd16_unit_chunks(int u, int ch) { return fwd16_unit_tiles(u) * ch + 1; }
__host__ __device__ constexpr int fwd16_unit_chunk_off(int u, int ch) { return fwd16_unit_tile_off(u) * ch + u; }
__host__ __device__ constexpr int fwd_unit_chunk_off(int u, int ch) { return fwd_unit_tile_off(u) * ch + u; }
__host__ __device__ constexpr int bwd_unit_chunks(int u, int ch) { return bwd_unit_tiles(u) * ch; }
__host__ __device__ constexpr int bwd_unit_chunk_off(int u, int ch) { return bwd_unit_tile_off(u) * ch; }
__host__ __device__ constexpr int bwd16_unit_chunks(int u, int ch) { return bwd16_unit_tiles(u) * ch; }
__host__ __device__ constexpr int bwd16_unit_chunk_off(int u, int ch) { return bwd16_unit_tile_off(u) * ch; }
__host__ __device__ constexpr int64_t total_chunks(int ch, int dir) {
  return dir == 0 ? (int64_t)FWD_TILES * ch + NUNIT_FWD
       : dir == 1 ? (int64_t)BWD_TILES * ch
       : dir == 2 ? (int64_t)FWD16_TILES * ch + NUNIT_FWD16
       : (int64_t)BWD16_TILES * ch;
}

struct ParamPtrs { const float* p[NPARAM]; };

// first chunk of every unit (+ the end), evaluated at compile time and passed by value:
// the unit of a chunk is then a scan of kernel arguments, not a runtime walk of the
// constexpr layout functions (which are loops)
struct UnitOffsets { int off[NUNIT_MAX + 1]; };
template <int CH, int DIR>
constexpr UnitOffsets unit_offsets() {
  UnitOffsets t{};
  const int nu = num_units(DIR);
  for (int u = 0; u <= nu; ++u)
    t.off[u] = DIR == 0 ? fwd_unit_chunk_off(u, CH) : DIR == 1 ? bwd_unit_chunk_off(u, CH)
             : DIR == 2 ? fwd16_unit_chunk_off(u, CH) : bwd16_unit_chunk_off(u, CH);
  return t;
}

// one thread per 16-B lane slot of one chunk
// The sources of packed lane-chunk i (chunk i >> 6, lane i & 63): weight(e, wp, idx, c) for each of its
// E elements (wp = -1: a zero element; else element idx of parameter wp, split part c of P::cvt_c), or, on
// a forward unit's bias chunk, bias(e, wp, idx) for its 4 fp32 values.
template <class P, int DIR, class Weight, class Bias>
__device__ __forceinline__ void pack_sources(int64_t i, const UnitOffsets& uo, Weight&& weight, Bias&& bias) {
  const int lane = (int)(i & 63);
  const int chunk = (int)(i >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int nunit = num_units(DIR);
  int u = 0;
  for (int k = 1; k < nunit; ++k) u += uo.off[k] <= chunk ? 1 : 0;
  const int within = chunk - uo.off[u];
  if constexpr (DIR == 2) {
    // 16-row unit (PBF3W, PF32W): lane l = r16 + 16 g holds weight row r16 of the unit, the E features
    // P::feat16(c, g, e) of K-block t, split part P::part16(c) (PBF3W: all 8 features of lane group g, chunk
    // c = 0 the hi, 1 the lo halves; PF32W: the 4 features 16 c + 4 g + e).  Bias chunk: lanes 0..3 hold
    // rows 4 lane + e (the accumulator's rows of lane group g = lane), rest zero.
    const int L = fwd16_unit_layer(u), m = u - fwd16_unit_first(L);
    const int w = fwd16_out_weight(L, m);
    if (within == fwd16_unit_tiles(u) * P::CH) {
      for (int e = 0; e < 4; ++e) {
        const int row = lane * 4 + e;
        const bool ok = lane < 4 && row < fwd16_out_valid(L, m);
        bias(e, ok ? w + 1 : -1, (int64_t)(fwd16_out_row0(L, m) + row));
      }
      return;
    }
    const int t = within / P::CH, c = within % P::CH, r16 = lane & 15, g = lane >> 4;
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int f = P::feat16(c, g, e);
      const bool ok = r16 < fwd16_out_valid(L, m) && f < fwd_in_valid(L, t);
      weight(e, ok ? w : -1,
             ok ? (int64_t)(fwd16_out_row0(L, m) + r16) * weight_K(w) + fwd_in_colbase(L, t) + f : (int64_t)0,
             P::part16(c));
    }
    return;
  }
  if constexpr (DIR == 3) {
    // 16-row dX unit (PF32W / PBF3W): half m & 1 of W^T output tile m >> 1 of stage s.  Lane l = r16 + 16 g holds
    // A[i][p] = W[p][i] for dX row i = the forward in-feature bwd_out_colbase + 16 (m & 1) + r16 and the E forward
    // out-features p = row0 + P::feat16(c, g, e) of input K-block t (forward output tile t of the stage's layer)
    const int s = bwd16_unit_stage(u), m = u - bwd16_unit_first(s), L = bwd_fwd_layer(s);
    const int t = within / P::CH, c = within % P::CH, r16 = lane & 15, g = lane >> 4;
    const int w = fwd_out_weight(L, t), i = bwd_out_colbase(s, m >> 1) + 16 * (m & 1) + r16;
#pragma unroll
    for (int e = 0; e < P::E; ++e) {
      const int f = P::feat16(c, g, e);
      const bool ok = f < fwd_out_valid(L, t);
      weight(e, ok ? w : -1, ok ? (int64_t)(fwd_out_row0(L, t) + f) * weight_K(w) + i : (int64_t)0, P::part16(c));
    }
    return;
  }
  if (DIR == 0 && within == fwd_unit_tiles(u) * P::CH) {
    // bias chunk: lanes 0..7 hold the 32 biases of the unit's output rows, rest zero
    const int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
    const int wp = fwd_out_weight(L, n);
    for (int e = 0; e < 4; ++e) {
      const int row = lane * 4 + e;
      const bool ok = lane < 8 && row < fwd_out_valid(L, n);
      bias(e, ok ? wp + 1 : -1, (int64_t)(fwd_out_row0(L, n) + row));
    }
    return;
  }
  const int t = within / P::CH, c = within % P::CH;
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int rho = P::rho_of(c, e);
    const int ar = acc_row(rho, h);
    int wp = -1;
    int64_t idx = 0;
    if (DIR == 0) {
      const int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
      const int w = fwd_out_weight(L, n);
      const int row = fwd_out_row0(L, n) + r, col = fwd_in_colbase(L, t) + ar;
      if (r < fwd_out_valid(L, n) && ar < fwd_in_valid(L, t)) wp = w, idx = (int64_t)row * weight_K(w) + col;
    } else {
      // A[i = forward in-feature (r)][p = forward out-feature of forward tile t (ar)]
      const int s = bwd_unit_stage(u), j = u - bwd_unit_first(s), L = bwd_fwd_layer(s);
      const int w = fwd_out_weight(L, t);
      const int row = fwd_out_row0(L, t) + ar, col = bwd_out_colbase(s, j) + r;
      if (ar < fwd_out_valid(L, t)) wp = w, idx = (int64_t)row * weight_K(w) + col;
    }
    weight(e, wp, idx, c);
  }
}

// direct pack (any parameter layout): one thread per lane-chunk, the sources walked on the device
template <class P, int DIR>
__global__ void pack_kernel(ParamPtrs prm, UnitOffsets uo, char* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total_chunks(P::CH, DIR) * 64) return;
  char* dst = out + i * 16;
  typename P::Store vals[P::E];
  bool is_bias = false;
  pack_sources<P, DIR>(
      i, uo,
      [&](int e, int wp, int64_t idx, int c) { vals[e] = P::cvt_c(wp < 0 ? 0.f : prm.p[wp][idx], c); },
      [&](int e, int wp, int64_t idx) {
        is_bias = true;
        ((float*)dst)[e] = wp < 0 ? 0.f : prm.p[wp][idx];
      });
  if (is_bias) return;
#pragma unroll
  for (int e = 0; e < P::E; ++e) ((typename P::Store*)dst)[e] = vals[e];
}

// Pack plan (r5): the sources of every packed element, built once per (policy, direction, device) by
// pack_plan_kernel, so that the per-step repack of a net whose 24 parameters lie back to back (FusedAdam's
// flat buffer) is one gather (pack_gather_kernel: ~30 instructions per lane-chunk instead of the ~2,000 of
// the unit / layer walk above, bit-identical).  Entry: bits 0-23 the element's offset in the net's flat
// parameters, bits 24-26 the split part c; PLAN_ZERO a zero element; PLAN_BIAS in entry E - 1 marks a
// bias lane-chunk whose entries 0-3 are fp32 values (E = 8 policies; fp32's E = 4 stores floats anyway).
constexpr uint32_t PLAN_ZERO = 0xFFFFFFFFu;
constexpr uint32_t PLAN_BIAS = 0xFE000000u;
template <class P, int DIR>
__global__ void pack_plan_kernel(UnitOffsets uo, uint32_t* plan) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total_chunks(P::CH, DIR) * 64) return;
  uint32_t* pl = plan + i * P::E;
  auto code = [](int wp, int64_t idx, int c) {
    return wp < 0 ? PLAN_ZERO : (uint32_t)(param_offset(wp) + idx) | ((uint32_t)c << 24);
  };
  bool is_bias = false;
  uint32_t ent[P::E];
  pack_sources<P, DIR>(
      i, uo, [&](int e, int wp, int64_t idx, int c) { ent[e] = code(wp, idx, c); },
      [&](int e, int wp, int64_t idx) {
        is_bias = true;
        ent[e] = code(wp, idx, 0);
      });
  if (is_bias)
    for (int e = 4; e < P::E; ++e) ent[e] = e == P::E - 1 ? PLAN_BIAS : PLAN_ZERO;
  for (int e = 0; e < P::E; ++e) pl[e] = ent[e];
}
template <class P>
__global__ void pack_gather_kernel(const float* __restrict__ flat, const uint32_t* __restrict__ plan, char* out,
                                   int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t ent[P::E];
#pragma unroll
  for (int q = 0; q < P::E / 4; ++q) {
    const uint4 v = ((const uint4*)(plan + i * P::E))[q];
    ent[4 * q] = v.x, ent[4 * q + 1] = v.y, ent[4 * q + 2] = v.z, ent[4 * q + 3] = v.w;
  }
  char* dst = out + i * 16;
  if (P::E == 8 && ent[P::E - 1] == PLAN_BIAS) {
    float f[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = ent[e] == PLAN_ZERO ? 0.f : flat[ent[e] & 0xFFFFFFu];
    *(float4*)dst = make_float4(f[0], f[1], f[2], f[3]);
    return;
  }
  typename P::Store vals[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e)
    vals[e] = P::cvt_c(ent[e] == PLAN_ZERO ? 0.f : flat[ent[e] & 0xFFFFFFu], (int)((ent[e] >> 24) & 7u));
  static_assert(sizeof(vals) == 16, "a lane-chunk is 16 bytes");
  *(uint4*)dst = __builtin_bit_cast(uint4, vals);
}

// ------------------------------------------------------------------------------------
// weight stream.  The packed units (one 32-row output tile of one layer, forward; one
// 32-row output tile of one dX stage, backward) are cut into GROUPS of consecutive units
// of one layer/stage that fit one LDS slot (<= SLOT_CAP KiB).  A 2-slot ring is filled by
// LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction) one group ahead, so a
// workgroup meets one barrier per group (4 hidden-layer units = 64 MFMAs per wave in
// bf16) instead of one per unit.
//
// The DMA is issued from inline asm, invisible to hipcc's waitcnt bookkeeping, and the
// group hand-off is a counted `s_waitcnt vmcnt(N)` + s_barrier where N = the vector-memory
// instructions this wave issued after the next group's DMA (the group's activation /
// gradient stores).  Loads, stores and LDS-DMA retire in issue order on one counter
// (MI355X_MICROARCH.md), so the wait covers the DMA and never the stores.  No
// compiler-visible global load may sit between a DMA and its wait (its compiler wait
// would drain the ring): all such loads are in the prologue.
// ------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;

// (NERF_DIAG_NO_DMA / NERF_DIAG_NO_STORE: diagnostic timing builds only -- the weight stream or
// the training stores left out, results meaningless -- to price them in the kernels' time)
#ifndef NERF_DIAG_NO_DMA
#define NERF_DIAG_NO_DMA 0
#endif
#ifndef NERF_DIAG_NO_STORE
#define NERF_DIAG_NO_STORE 0
#endif
// (NERF_DIAG_NO_MASK / NERF_DIAG_NO_ACT: the wide forward without its mask bits / without its activation stores)
#ifndef NERF_DIAG_NO_MASK
#define NERF_DIAG_NO_MASK 0
#endif
#ifndef NERF_DIAG_NO_ACT
#define NERF_DIAG_NO_ACT 0
#endif
// (NERF_DIAG_STAMPS: diagnostic only -- the forward overwrites two raw rows per workgroup with its CU id and
// entry / prologue-done / end timestamps, tools/wg_stamps.py)
#ifndef NERF_DIAG_STAMPS
#define NERF_DIAG_STAMPS 0
#endif
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t lds_wave_base) {
  if constexpr (NERF_DIAG_NO_DMA) return;
  uint32_t saved;  // m0 is reserved to the compiler: save and restore it around the DMA
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_wave_base)) : "memory");
}

// every younger-than-N vector memory op of this wave may still be in flight; all LDS ops
// done; then the workgroup barrier.  "memory": no LDS/global access crosses it.
template <int N>
__device__ __forceinline__ void wait_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// hand a loaded value to an empty asm right after a prologue wait: hipcc then places its
// own wait for the load there (already satisfied) instead of at the first use in the main
// loop, where it would also drain the in-flight weight DMA
__device__ __forceinline__ void settle(float& x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void settle(uint32_t& x) { asm volatile("" : "+v"(x)); }

template <int... I, class F>
__device__ __forceinline__ void sfor_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
// compile-time unrolled loop: f(std::integral_constant<int, i>) for i in [0, N)
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(std::make_integer_sequence<int, N>{}, f);
}

__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }

// (a 3-slot ring of 48 KiB slots, DMA two groups ahead, measured slower everywhere in round 4:
// profiles/r4/pipeline_experiments.json)
constexpr int NSLOT = 2;       // ring slots; the DMA runs one group ahead
constexpr int SLOT_CAP = 72;   // KiB (1 KiB chunks) per slot: 144 KiB of the 160 KiB LDS
constexpr int PF = NSLOT - 1;
constexpr int GROUP_MAX = 8;   // units per group
#ifndef NERF_GROUP_ACROSS
#define NERF_GROUP_ACROSS 1    // groups may span layers: every group fills its slot
#endif

struct Group { int u0, n, c0, nch; };  // first unit, units, first chunk, chunks

// DIR 0: forward units (DENSITY: trunk + alpha only, occupancy_grid.py:60 reads raw[...,3]);
// DIR 1: dX-chain units; DIR 2: 16-row forward units (PBF3W)
template <int DIR, bool DENSITY>
__host__ __device__ constexpr bool unit_used(int u) {
  return DIR == 1 || DIR == 3 || !DENSITY ||
         (DIR == 0 ? (u < fwd_unit_first(LFA) || u == fwd_unit_first(LFA) + 8)
                   : (u < fwd16_unit_first(LFA) || u == fwd16_unit_first(LFA) + 16));
}
template <int DIR> __host__ __device__ constexpr int unit_seg(int u) {
  return DIR == 0 ? fwd_unit_layer(u) : DIR == 1 ? bwd_unit_stage(u) : DIR == 2 ? fwd16_unit_layer(u) : bwd16_unit_stage(u);
}
template <int DIR> __host__ __device__ constexpr int unit_chunks(int u, int ch) {
  return DIR == 0 ? fwd_unit_chunks(u, ch) : DIR == 1 ? bwd_unit_chunks(u, ch)
       : DIR == 2 ? fwd16_unit_chunks(u, ch) : bwd16_unit_chunks(u, ch);
}
template <int DIR> __host__ __device__ constexpr int unit_chunk_off(int u, int ch) {
  return DIR == 0 ? fwd_unit_chunk_off(u, ch) : DIR == 1 ? bwd_unit_chunk_off(u, ch)
       : DIR == 2 ? fwd16_unit_chunk_off(u, ch) : bwd16_unit_chunk_off(u, ch);
}

// greedy grouping: consecutive used units of one segment while the slot has room
template <int DIR, bool DENSITY, int CH>
struct Groups {
  Group g[NUNIT_MAX];
  int n;
  __host__ __device__ constexpr Groups() : g(), n(0) {
    const int NU = num_units(DIR);
    int u = 0;
    while (u < NU) {
      if (!unit_used<DIR, DENSITY>(u)) {
        ++u;
        continue;
      }
      Group G{u, 0, unit_chunk_off<DIR>(u, CH), 0};
      const int seg = unit_seg<DIR>(u);
      while (u < NU && unit_used<DIR, DENSITY>(u) && (NERF_GROUP_ACROSS || unit_seg<DIR>(u) == seg) &&
             G.n < GROUP_MAX &&
             G.nch + unit_chunks<DIR>(u, CH) <= SLOT_CAP) {
        G.nch += unit_chunks<DIR>(u, CH);
        ++G.n;
        ++u;
      }
      g[n++] = G;
    }
  }
};
template <int DIR, bool DENSITY, int CH>
struct GroupTable {
  static constexpr Groups<DIR, DENSITY, CH> t{};
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4 lds_cu4;
__device__ __forceinline__ uint4 as_uint4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

// per-lane LDS base of a unit's chunks (lane-linear: + 16 lane bytes), laundered through
// an empty asm: every read of the unit is then this one VGPR + an immediate offset
// (< 64 KiB).  Left visible, hipcc materialises one address VGPR per distinct chunk offset
// of both ring slots and keeps them all live across the unrolled kernel.
__device__ __forceinline__ lds_cu4* lds_ptr(uint32_t byte_addr) {
  settle(byte_addr);
  return (lds_cu4*)(uintptr_t)byte_addr;
}

// The MFMA steps of a group as one flat compile-time list: step k = (unit j of the group,
// input tile t, chunk c), in execution order.  A group's body is straight-line code over
// it with the A operand (weights, LDS) prefetched PD steps ahead across unit boundaries
// -- hipcc on its own keeps one ds_read in flight and waits lgkmcnt(0) before every MFMA.

// DMA wave-instructions (1 KiB global_load_lds each) per wave for group g (fetch_group)
template <class P, int DIR, bool DENSITY>
__host__ __device__ constexpr int group_dma_units(int g) {
  return (GroupTable<DIR, DENSITY, P::CH>::t.g[g].nch + P::WAVES - 1) / P::WAVES;
}
template <class P, int DIR, bool DENSITY>
__host__ __device__ constexpr int group_dma(int g) {
  return group_dma_units<P, DIR, DENSITY>(g);
}
// vmcnt of the hand-off at the end of group g (group g + 1's DMA must have landed): the
// wave's vector-memory ops younger than that DMA = the DMAs of groups g + 2 .. g + PF and
// the stores of the iterations g + 1 - PF .. g (each issued after its iteration's DMA), plus
// the prologue's stores when group g + 1 was fetched in the prologue.
template <class P, int DIR, bool DENSITY, class StoresFn>
__host__ __device__ constexpr int handoff_vmcnt(int g, StoresFn stores, int prologue_stores) {
  const int NG = GroupTable<DIR, DENSITY, P::CH>::t.n;
  int n = 0;
  for (int j = g + 2; j <= g + PF && j < NG; ++j) n += group_dma<P, DIR, DENSITY>(j);
  for (int i = (g + 1 - PF > 0 ? g + 1 - PF : 0); i <= g; ++i) n += stores(i);
  if (g + 1 < PF) n += prologue_stores;
  return n;
}

struct Step { int j, u, t, c, off, kin, len; bool first, last; };
template <int DIR> __host__ __device__ constexpr int unit_tiles(int u) {
  return DIR == 0 ? fwd_unit_tiles(u) : DIR == 1 ? bwd_unit_tiles(u) : DIR == 2 ? fwd16_unit_tiles(u) : bwd16_unit_tiles(u);
}
template <int DIR, bool DENSITY, int CH>
__host__ __device__ constexpr int group_steps(int g) {
  const Group G = GroupTable<DIR, DENSITY, CH>::t.g[g];
  int n = 0;
  for (int j = 0; j < G.n; ++j) n += unit_tiles<DIR>(G.u0 + j) * CH;
  return n;
}
template <int DIR, bool DENSITY, int CH>
__host__ __device__ constexpr Step group_step(int g, int k) {
  const Group G = GroupTable<DIR, DENSITY, CH>::t.g[g];
  for (int j = 0; j < G.n; ++j) {
    const int u = G.u0 + j, n = unit_tiles<DIR>(u) * CH;
    if (k < n) {
      const int t = k / CH, c = k % CH;
      return Step{j, u, t, c, unit_chunk_off<DIR>(u, CH) - G.c0 + k, k, n, k == 0, k == n - 1};
    }
    k -= n;
  }
  return Step{-1, -1, 0, 0, 0, 0, 0, false, false};
}
// A-operand prefetch distance in steps (a bf16 step is one 32-cycle MFMA, an fp32 step four
// 64-cycle ones) and how many steps into unit j + 1 the finish of unit j is issued (its
// VALU then interleaves with unit j + 1's MFMAs instead of stalling the wave)
#ifndef NERF_PREFETCH_BF16
#define NERF_PREFETCH_BF16 3
#endif
#ifndef NERF_PREFETCH_F32
#define NERF_PREFETCH_F32 2  // (fp32 training forward 4.99 / 4.94 / 5.08 ms at 1 / 2 / 3 steps ahead)
#endif
#ifndef NERF_FINISH_DELAY
#define NERF_FINISH_DELAY 3
#endif
#ifndef NERF_PREFETCH_F32W
#define NERF_PREFETCH_F32W 2  // (a PF32W step is four 32-cycle MFMAs)
#endif
template <class P> __host__ __device__ constexpr int prefetch_depth() {
  return P::KIND == K_F32 ? NERF_PREFETCH_F32 : P::KIND == K_F32W ? NERF_PREFETCH_F32W : NERF_PREFETCH_BF16;  // a bf16 / bf16x3 step is 1-2 short MFMAs
}
constexpr int FINISH_DELAY = NERF_FINISH_DELAY;
// (the wide bf16 dX, one chunk per K-block: the dX stage bV reads bRGB's last output K-block at its step 3, so its
// finish runs 1 step into bV's first unit -- with 3 FinishSchedule refuses the build)
#ifndef NERF_FINISH_DELAY_BF16W
#define NERF_FINISH_DELAY_BF16W 1
#endif

// Cross-group finish: the last unit of a group is finished after the barrier.  Not in the
// bf16x3 forward: a finished accumulator carried over the barrier (plus the hi / lo split of
// the finish) takes it past 512 VGPRs (139 spilled); finished in-group it needs none.
// (r5: with the lean DMA and packed masks the bf16x3 forward fits cross-group finish without spills, 372
// VGPRs, but it is not faster: bf16x3f training forward 1.609 vs 1.599 ms)
template <class P, int DIR> __host__ __device__ constexpr bool cross_finish() {
  return !(P::KIND == K_BF16X3 && DIR == 0);
}
// the unit finished inside group g: (first, last] = units whose finish is issued in g.
// With cross_finish() the last unit of a group is finished FINISH_DELAY steps into the
// next group (after the barrier), so no group ends in a VALU burst that every wave of the
// workgroup runs at once; its stores then count against the next group's hand-off.
template <int DIR, bool DENSITY, int CH, bool CROSS>
__host__ __device__ constexpr bool finished_in_group(int g, int u) {
  const auto& T = GroupTable<DIR, DENSITY, CH>::t;
  const Group G = T.g[g];
  const int last = G.u0 + G.n - 1;
  if (!CROSS) return u >= G.u0 && u <= last;
  const bool prev = g > 0 && u == T.g[g - 1].u0 + T.g[g - 1].n - 1;
  return prev || (u >= G.u0 && (u < last || (u == last && g + 1 == T.n)));
}

// Finish parts.  A unit's epilogue (ReLU, mask bits, pack / hi-lo split, stores: ~60-110
// instructions) issued as one run stalls the matrix pipe of a one-wave-per-SIMD kernel (fp32,
// bf16x3) for the whole run: nothing else feeds it (the gfx950 assembly of the bf16x3
// training forward had 70 % of its non-MFMA instructions in 138 runs of > 20 between two
// MFMAs).  With NP parts, part p (register pairs [8p/NP, 8(p+1)/NP)) is issued FINISH_DELAY + p
// steps into the next unit, clamped to that unit's last step; the last part stores.
// Any value is checked at compile time: FinishSchedule (below) static_asserts that no MFMA reads a tile pair
// before the part that writes it.  (Round 5 saw NERF_FINISH_PARTS_BF16 = 2 / 8 write masks / dZ that differed
// run to run.  Parts 8 is that clamping hazard and no longer compiles; parts 2 was an inline-asm VGPR write
// racing an MFMA write-back (nonzero_bf16x2), fixed for every placement.  Round 6, tools/race_diag.py,
// profiles/r6/race_diag_*.json: bf16 parts 2 / 4 and bf16x3 parts 4 / 8 bit-identical, run to run and to
// each other.)
#ifndef NERF_FINISH_PARTS_F32
#define NERF_FINISH_PARTS_F32 1  // (fp32: 8 parts + spread DMA measured 4.88 -> 5.05 ms, training forward)
#endif
#ifndef NERF_FINISH_PARTS_BF16
#define NERF_FINISH_PARTS_BF16 4  // with NERF_DMA_SPREAD_BF16 3: bf16 inference forward 0.517 -> 0.488 ms,
#endif                            // dX 0.619 -> 0.609 at 524,288 samples (r4; 8 parts: no gain)
#ifndef NERF_FINISH_PARTS_BF3
#define NERF_FINISH_PARTS_BF3 8  // with NERF_DMA_SPREAD_BF3 3: bf16x3 forward 1.70 -> 1.58 ms, training
#endif                           // forward 1.97 -> 1.88, dX 1.73 -> 1.65 at 524,288 samples (r4)
#ifndef NERF_FINISH_PARTS_BF3W
#define NERF_FINISH_PARTS_BF3W 2  // (a 16x16 tile's 2 register pairs)
#endif
#ifndef NERF_FINISH_PARTS_F32W
#define NERF_FINISH_PARTS_F32W 2
#endif
#ifndef NERF_FINISH_PARTS_BF16W
#define NERF_FINISH_PARTS_BF16W 2
#endif
template <class P> __host__ __device__ constexpr int finish_parts() {
  return P::KIND == K_F32 ? NERF_FINISH_PARTS_F32 : P::KIND == K_BF16 ? NERF_FINISH_PARTS_BF16
       : P::KIND == K_BF16X3W ? NERF_FINISH_PARTS_BF3W : P::KIND == K_F32W ? NERF_FINISH_PARTS_F32W
       : P::KIND == K_BF16W ? NERF_FINISH_PARTS_BF16W : NERF_FINISH_PARTS_BF3;
}
// DMA spread.  0: the next group's LDS-DMA pieces (up to 18 per wave, ~7 instructions each)
// are issued as one burst at the group's start; S > 0: piece i at step i (NS / S) / NF of the
// group's NS steps, i.e. inside the first 1/S of the group (they must land before its end).
#ifndef NERF_DMA_SPREAD_F32
#define NERF_DMA_SPREAD_F32 0
#endif
#ifndef NERF_DMA_SPREAD_BF16
#define NERF_DMA_SPREAD_BF16 3
#endif
#ifndef NERF_DMA_SPREAD_BF3
#define NERF_DMA_SPREAD_BF3 3
#endif
#ifndef NERF_DMA_SPREAD_BF3W
#define NERF_DMA_SPREAD_BF3W 3
#endif
#ifndef NERF_DMA_SPREAD_F32W
#define NERF_DMA_SPREAD_F32W 3
#endif
#ifndef NERF_DMA_SPREAD_BF16W
#define NERF_DMA_SPREAD_BF16W 3
#endif
template <class P> __host__ __device__ constexpr int dma_spread() {
  return PF != 1 ? 0 : P::KIND == K_F32 ? NERF_DMA_SPREAD_F32 : P::KIND == K_BF16 ? NERF_DMA_SPREAD_BF16
       : P::KIND == K_BF16X3W ? NERF_DMA_SPREAD_BF3W : P::KIND == K_F32W ? NERF_DMA_SPREAD_F32W
       : P::KIND == K_BF16W ? NERF_DMA_SPREAD_BF16W : NERF_DMA_SPREAD_BF3;
}

// step (in group g) at which part p of unit u's finish is issued, or -1 when u is not
// finished in g
template <class P, int DIR, bool DENSITY>
__host__ __device__ constexpr int part_step(int g, int u, int p) {
  const auto& T = GroupTable<DIR, DENSITY, P::CH>::t;
  const Group G = T.g[g];
  if (!finished_in_group<DIR, DENSITY, P::CH, cross_finish<P, DIR>()>(g, u)) return -1;
  const int NS = group_steps<DIR, DENSITY, P::CH>(g);
  if (u == G.u0 + G.n - 1) return NS - 1;  // the group's last unit, finished in-group: at its last step
  const int js = u < G.u0 ? 0 : u - G.u0 + 1;  // the unit after u (this group's first, or u + 1)
  int start = 0;
  for (int j = 0; j < js; ++j) start += unit_tiles<DIR>(G.u0 + j) * P::CH;
  const int len = unit_tiles<DIR>(G.u0 + js) * P::CH;
  const int d = (P::KIND == K_BF16W ? NERF_FINISH_DELAY_BF16W : FINISH_DELAY) + p;
  return start + (d < len - 1 ? d : len - 1);
}
// step (in group g) of the i-th of the next group's NF DMA pieces (dma_spread > 0)
template <class P, int DIR, bool DENSITY>
__host__ __device__ constexpr int dma_piece_step(int g, int i) {
  const int NS = group_steps<DIR, DENSITY, P::CH>(g);
  const int NF = group_dma_units<P, DIR, DENSITY>(g + 1);
  const int front = (NS + dma_spread<P>() - 1) / dma_spread<P>();
  return i * front / NF;
}
// vmcnt of the hand-off at the end of group g when the next group's DMA is spread over
// group g: the stores issued at or after the step of its last piece (a step issues its DMA
// pieces first, then its MFMAs, then any finish parts)
template <class P, int DIR, bool DENSITY, class StoresFn>
__host__ __device__ constexpr int handoff_vmcnt_spread(int g, StoresFn unit_stores) {
  if (g + 1 >= GroupTable<DIR, DENSITY, P::CH>::t.n) return 0;  // (the last group: no hand-off)
  const int last = dma_piece_step<P, DIR, DENSITY>(g, group_dma_units<P, DIR, DENSITY>(g + 1) - 1);
  const int NU = num_units(DIR);
  int n = 0;
  for (int u = 0; u < NU; ++u) {
    const int s = part_step<P, DIR, DENSITY>(g, u, finish_parts<P>() - 1);
    if (s >= last) n += unit_stores(u);
  }
  return n;
}

// ------------------------------------------------------------------------------------
// Register tile slots and the finish-schedule check (r6).
//
// A wave's B-operand tiles live in registers: the activation / gradient ping-pong arrays Ha[0..7]
// and Hb[0..7], the encodings X[0..1] and D (forward) and the output-gradient seeds G and DA (dX).
// Every unit reads its input tiles from slots and its finish parts write its output tile, pair by
// pair, IN PLACE into a slot -- which the next layer's first unit reads.  The two tables below
// are the kernels' own (FwdWave::in_tile / DxWave::in_tile and the finishes go through them), so
// the schedule model below checks the code that runs.
//
// The race found in round 5 (bf16 finish parts 2 / 8: masks / dZ that differed between two runs
// of one launch) is this hand-off.  A finish part is issued FINISH_DELAY + p steps into the next
// unit, CLAMPED to that unit's last step, and within a step the finish runs after the MFMA.
// Where the next unit has few input tiles -- LRGB after LV (4 tiles), the dX stage bV after
// bRGB (4 tiles) -- eight parts land at steps 3..7 of an 8-step unit, and the parts writing
// pairs 3..7 of tile 3 come after the MFMAs that read them (steps 6 and 7).  Those MFMAs read the
// slot's OLD registers: in the forward the previous layer's values (deterministic, wrong), in the
// dX chain Hb[3] before its first write (uninitialised registers: different on every run).  The
// ISA-level hand-off check could not see it: it is a register dependence the program order
// itself gets wrong, not a memory-counter one.  finish_schedule_ok() below simulates every
// group's steps and fails the build of any placement where an MFMA reads a pair before its
// producer's part (or a later producer's part overwrites it first), or a part reads `pend` after
// it was reassigned.
// ------------------------------------------------------------------------------------
enum TileSlot { TS_HA = 0, TS_HB = 8, TS_X = 16, TS_D = 18, TS_G = 19, TS_DA = 20, TS_NONE = -1 };
__host__ __device__ constexpr bool finish_slot(int s) { return s >= TS_HA && s < TS_X; }  // written by finishes
// forward layer L: input tile t, output tile n
__host__ __device__ constexpr int fwd_in_slot(int L, int t) {
  return L == L0 ? TS_X + t
       : L == L5 ? (t < 2 ? TS_X + t : TS_HA + t - 2)
       : L == LV ? (t < 8 ? TS_HA + t : (int)TS_D)
       : L == LRGB ? TS_HB + t
       : (L == L1 || L == L3 || L == L7) ? TS_HA + t
       : TS_HB + t;  // L2, L4, L6, LFA
}
__host__ __device__ constexpr int fwd_out_slot(int L, int n) {
  return L == LRGB || (L == LFA && n == 8) ? (int)TS_NONE  // (rgb / alpha: scalars)
       : (L == L0 || L == L2 || L == L4 || L == L6 || L == LFA) ? TS_HA + n
       : TS_HB + n;  // L1, L3, L5, L7, LV
}
// dX stage s: input tile t, output tile j
__host__ __device__ constexpr int bwd_in_slot(int s, int t) {
  return s == B_RGB ? (int)TS_G
       : s == B_V ? TS_HB + t
       : s == B_FA ? (t < 8 ? TS_HA + t : (int)TS_DA)
       : (s == B_7 || s == B_5 || s == B_3 || s == B_1) ? TS_HB + t
       : TS_HA + t;  // B_6, B_4, B_2
}
__host__ __device__ constexpr int bwd_out_slot(int s, int j) {
  return (s == B_RGB || s == B_FA || s == B_6 || s == B_4 || s == B_2) ? TS_HB + j : TS_HA + j;
}
template <int DIR> __host__ __device__ constexpr int unit_in_slot(int u, int t) {
  return DIR == 0 ? fwd_in_slot(fwd_unit_layer(u), t)
       : DIR == 1 ? bwd_in_slot(bwd_unit_stage(u), t)
       : DIR == 2 ? fwd_in_slot(fwd16_unit_layer(u), t)
       : bwd_in_slot(bwd16_unit_stage(u), t);
}
// 16-row unit (DIR 2): output tile m fills half m & 1 (elements 4 (m & 1) .. + 3) of K-block slot m >> 1
template <int DIR> __host__ __device__ constexpr int unit_out_slot(int u) {
  return DIR == 0 ? fwd_out_slot(fwd_unit_layer(u), u - fwd_unit_first(fwd_unit_layer(u)))
       : DIR == 1 ? bwd_out_slot(bwd_unit_stage(u), u - bwd_unit_first(bwd_unit_stage(u)))
       : DIR == 2 ? fwd_out_slot(fwd16_unit_layer(u), (u - fwd16_unit_first(fwd16_unit_layer(u))) >> 1)
       : bwd_out_slot(bwd16_unit_stage(u), (u - bwd16_unit_first(bwd16_unit_stage(u))) >> 1);
}
// the register pairs of its slot a unit's finish writes (a 32x32 tile: all 8; a 16-row unit: 2 of a K-block's 4)
template <int DIR> __host__ __device__ constexpr int unit_out_pairs(int u) {
  return DIR == 2 ? (((u - fwd16_unit_first(fwd16_unit_layer(u))) & 1) ? 0xC : 0x3)
       : DIR == 3 ? (((u - bwd16_unit_first(bwd16_unit_stage(u))) & 1) ? 0xC : 0x3) : 0xFF;
}
// register pairs (bit k = registers 2k, 2k + 1) of a tile that MFMA chunk c reads / finish part p writes
template <class P> __host__ __device__ constexpr int chunk_pairs(int c) {
  int m = 0;
  for (int e = 0; e < P::E; ++e) {
    const int rho = P::rho_of(c, e);
    if (rho < 16) m |= 1 << (rho >> 1);
  }
  return m;
}
// pairs of an output tile: 8 (32x32 accumulator, 16 registers), 2 (16x16, 4 registers)
template <class P> __host__ __device__ constexpr int tile_pairs() { return wide_kind<P>() ? 2 : 8; }
template <class P> __host__ __device__ constexpr int part_pairs(int p) {
  constexpr int NP = finish_parts<P>(), TP = tile_pairs<P>();
  int m = 0;
  for (int k = TP * p / NP; k < TP * (p + 1) / NP; ++k) m |= 1 << k;
  return m;
}
// the pairs of its slot part p of unit u writes
template <class P, int DIR> __host__ __device__ constexpr int part_write_pairs(int u, int p) {
  return DIR < 2 ? part_pairs<P>(p) : part_pairs<P>(p) << (unit_out_pairs<DIR>(u) == 0xC ? 2 : 0);
}
// Positions in the straight-line schedule: 4 * (global step) + phase, the phases of one step in
// group_body's order: 0 DMA pieces, 1 pend / init + MFMA, 2 the previous unit's finish parts, 3 the
// group's last unit (finished in-group, or parked in `pend` for the next group).
// finish_schedule_violation() is 0 when the schedule is sound; else a code naming the first
// violation: 1 an MFMA reads a pair before its producer's part writes it (or reads a slot no unit
// wrote), 2 a later producer's part overwrites the pair before the read, 3 a part reads `pend`
// after it was reassigned, 4 a finish part is never issued.
template <class P, int DIR, bool DENSITY>
struct FinishSchedule {
  static constexpr int NU = num_units(DIR);
  static constexpr int NP = finish_parts<P>();
  int pos[NUNIT_MAX][8];   // position of part p of unit u (-1: none)
  int pend_at[NUNIT_MAX];  // position at which `pend` takes unit u (-1)
  int violation;
  __host__ __device__ constexpr FinishSchedule() : pos(), pend_at(), violation(0) {
    const auto& T = GroupTable<DIR, DENSITY, P::CH>::t;
    for (int u = 0; u < NU; ++u) {
      pend_at[u] = -1;
      for (int p = 0; p < 8; ++p) pos[u][p] = -1;
    }
    int base = 0;
    for (int g = 0; g < T.n; ++g) {
      const Group G = T.g[g];
      const int NS = group_steps<DIR, DENSITY, P::CH>(g);
      const int last = G.u0 + G.n - 1;
      // units finished in g: the previous group's last unit (cross-group finish) and G's own
      for (int u = (g > 0 ? T.g[g - 1].u0 + T.g[g - 1].n - 1 : G.u0); u <= last; ++u)
        for (int p = 0; p < NP; ++p) {
          const int st = part_step<P, DIR, DENSITY>(g, u, p);
          if (st >= 0) pos[u][p] = 4 * (base + st) + (u == last ? 3 : 2);
        }
      for (int j = 1, k = unit_tiles<DIR>(G.u0) * P::CH; j < G.n; k += unit_tiles<DIR>(G.u0 + j) * P::CH, ++j)
        pend_at[G.u0 + j - 1] = 4 * (base + k) + 1;  // (the first step of unit j)
      if (!finished_in_group<DIR, DENSITY, P::CH, cross_finish<P, DIR>()>(g, last)) pend_at[last] = 4 * (base + NS - 1) + 3;
      base += NS;
    }
    violation = check();
  }
  __host__ __device__ constexpr int check() const {
    const auto& T = GroupTable<DIR, DENSITY, P::CH>::t;
    int out[NUNIT_MAX] = {}, opairs[NUNIT_MAX] = {}, pw[NUNIT_MAX][8] = {}, next_w[NUNIT_MAX][8] = {};
    int ntiles[NUNIT_MAX] = {}, in_slot[NUNIT_MAX][10] = {};  // (precomputed: the unit walks are loops)
    for (int u = 0; u < NU; ++u) {
      ntiles[u] = unit_tiles<DIR>(u);
      for (int t = 0; t < ntiles[u]; ++t) in_slot[u][t] = unit_in_slot<DIR>(u, t);
      out[u] = unit_used<DIR, DENSITY>(u) ? unit_out_slot<DIR>(u) : (int)TS_NONE;
      opairs[u] = finish_slot(out[u]) ? unit_out_pairs<DIR>(u) : 0;
      for (int p = 0; p < NP; ++p) pw[u][p] = part_write_pairs<P, DIR>(u, p);
    }
    {  // next_w[u][q]: the next unit after u that writes pair q of u's slot (-1: none)
      int seen[TS_X][8] = {};
      for (int sl = 0; sl < TS_X; ++sl)
        for (int q = 0; q < 8; ++q) seen[sl][q] = -1;
      for (int u = NU - 1; u >= 0; --u)
        for (int q = 0; q < 8; ++q) {
          next_w[u][q] = -1;
          if ((opairs[u] >> q) & 1) {
            next_w[u][q] = seen[out[u]][q];
            seen[out[u]][q] = u;
          }
        }
    }
    for (int u = 0; u < NU; ++u) {
      if (!unit_used<DIR, DENSITY>(u)) continue;
      for (int p = 0; p < NP; ++p) {
        if (pos[u][p] < 0) return 4;
        if ((pos[u][p] & 3) == 3) continue;  // finished in-group from `acc`
        // `pend` holds u from pend_at[u] until the next unit's assignment
        if (pend_at[u] < 0 || pend_at[u] >= pos[u][p]) return 3;
        for (int v = u + 1; v < NU; ++v)
          if (pend_at[v] >= 0 && pend_at[v] < pos[u][p]) return 3;
      }
    }
    // writer[slot][pair]: the last unit (in unit order, before the reading unit) that writes the pair
    int writer[TS_X][8] = {};
    for (int sl = 0; sl < TS_X; ++sl)
      for (int q = 0; q < 8; ++q) writer[sl][q] = -1;
    int base = 0, done = 0;  // (writer holds the units < done, in unit order)
    for (int g = 0; g < T.n; ++g) {
      const Group G = T.g[g];
      for (int j = 0; j < G.n; ++j) {
        const int u = G.u0 + j;
        for (; done < u; ++done)
          for (int q = 0; q < 8; ++q)
            if ((opairs[done] >> q) & 1) writer[out[done]][q] = done;
        const int nt = ntiles[u];
        for (int t = 0; t < nt; ++t) {
          const int slot = in_slot[u][t];
          if (!finish_slot(slot)) {
            base += P::CH;
            continue;
          }
          for (int c = 0; c < P::CH; ++c, ++base) {
            const int rpos = 4 * base + 1, cp = chunk_pairs<P>(c);
            for (int q = 0; q < 8; ++q) {
              if (!((cp >> q) & 1)) continue;
              const int prod = writer[slot][q];
              if (prod < 0) return 1;
              const int nv = next_w[prod][q];
              for (int p = 0; p < NP; ++p) {
                if (((pw[prod][p] >> q) & 1) && pos[prod][p] >= rpos) return 1;
                // the next unit writing the pair must not write it before this read
                if (nv >= 0 && ((pw[nv][p] >> q) & 1) && pos[nv][p] >= 0 && pos[nv][p] < rpos) return 2;
              }
            }
          }
        }
      }
    }
    return 0;
  }
};
template <class P, int DIR, bool DENSITY> __host__ __device__ constexpr int finish_schedule_violation() {
  return FinishSchedule<P, DIR, DENSITY>{}.violation;
}

// W: the wave object; it provides in_tile<u, t>(), prefetch<u>() (issue unit u's side
// reads one unit ahead), init<u>(acc) (initial accumulator), finish_part<u, p>(acc),
// fetch_piece<g, i>() (the i-th DMA piece of group g) and a pending accumulator `pend` that
// carries a finished chain to its deferred finish
template <class P, int DIR, bool DENSITY, int g, class W>
__device__ __forceinline__ void group_body(W& w, lds_cu4* wl) {
  constexpr int NS = group_steps<DIR, DENSITY, P::CH>(g);
  constexpr int PDP = prefetch_depth<P>();
  constexpr int NP = finish_parts<P>();
  constexpr auto& T = GroupTable<DIR, DENSITY, P::CH>::t;
  constexpr Group G = T.g[g];
  constexpr int PREV_U = g > 0 ? T.g[g - 1].u0 + T.g[g - 1].n - 1 : -1;  // previous group's last unit
  constexpr bool SPREAD = dma_spread<P>() > 0 && g + 1 < T.n;
  constexpr int NF = SPREAD ? group_dma_units<P, DIR, DENSITY>(g + 1) : 0;
  uint4 ring[PDP];
  sfor<(NS < PDP ? NS : PDP)>([&](auto kk) {
    constexpr int k = decltype(kk)::value;
    constexpr Step S = group_step<DIR, DENSITY, P::CH>(g, k);
    ring[k] = as_uint4(wl[S.off * 64]);
  });
  w.template prefetch<G.u0>();
  typename P::Acc acc;
  sfor<NS>([&](auto kk) {
    constexpr int k = decltype(kk)::value;
    constexpr Step S = group_step<DIR, DENSITY, P::CH>(g, k);
    if constexpr (SPREAD) {
      sfor<NF>([&](auto ii) {
        if constexpr (dma_piece_step<P, DIR, DENSITY>(g, decltype(ii)::value) == k)
          w.template fetch_piece<g + 1, decltype(ii)::value>();
      });
    }
    const uint4 a = ring[k % PDP];
    if constexpr (k + PDP < NS) {
      constexpr Step N = group_step<DIR, DENSITY, P::CH>(g, k + PDP);
      ring[k % PDP] = as_uint4(wl[N.off * 64]);
    }
    if constexpr (S.first) {
      if constexpr (S.j > 0) w.pend = acc;
      w.template init<S.u>(acc);
      if constexpr (S.j + 1 < G.n) w.template prefetch<S.u + 1>();
    }
    acc = P::mma(a, w.template in_tile<S.u, S.t>(), S.c, acc);
    constexpr int U_BEFORE = S.j > 0 ? S.u - 1 : PREV_U;
    if constexpr (U_BEFORE >= 0) {
      sfor<NP>([&](auto pp) {
        if constexpr (part_step<P, DIR, DENSITY>(g, U_BEFORE, decltype(pp)::value) == k)
          w.template finish_part<U_BEFORE, decltype(pp)::value>(w.pend);
      });
    }
    if constexpr (S.last && S.j == G.n - 1) {
      if constexpr (finished_in_group<DIR, DENSITY, P::CH, cross_finish<P, DIR>()>(g, S.u))
        sfor<NP>([&](auto pp) { w.template finish_part<S.u, decltype(pp)::value>(acc); });
      else w.pend = acc;
    }
  });
}

// DMA piece i of a wave for a group of NCH chunks starting at chunk C0 into slot `slot_base`:
// every wave issues exactly group_dma_units pieces (the last chunk is re-copied by the surplus
// waves -- identical bytes), so the count a later wait needs is a compile-time constant
template <class P, int C0, int NCH, int I, bool LAUNDER = false>
__device__ __forceinline__ void fetch_piece(const uint4* gsrc, uint32_t slot_base, int wave, int lane) {
  if constexpr (LAUNDER) {  // (persistent forward: the chunk indices are recomputed per group, not
    uint32_t w = wave;      // CSE'd across the groups and held -- spilled -- across the block loop)
    settle(w);
    wave = (int)w;
  }
  const int k = cmin(wave + P::WAVES * I, NCH - 1);
  glds16_asm(gsrc + (int64_t)(C0 + k) * 64 + lane, slot_base + (uint32_t)k * 1024u);
}

// Lean form of the same piece (NERF_DMA_LEAN).  Wave w's piece I is chunk w + WAVES I, so with the
// per-lane VGPR vlane = 16 lane + 1024 w and the wave-uniform swave = LDS base + 1024 w held for the
// whole kernel, the piece's global offset and LDS address are those plus compile-time constants:
// `s_add_u32 m0` (the LDS destination), `s_nop 0` (the wait state an M0 write needs before an
// LDS-DMA) and the DMA in the SADDR form on the packed-weight base; the per-lane offset vlane + GOFF is
// a v_add_u32 that hipcc places itself (4 instructions per piece; round 5 put the v_add_u32 inside
// the asm, as the m0 wait state, for 3).  Round 6: no VGPR is written inside inline asm any more --
// hipcc's hazard recognizer does not cover an asm VGPR write that lands on a register an in-flight
// MFMA still writes or reads as SrcC (the mask race, nonzero_bf16x2 above); a compiler-placed
// v_add_u32 gets its wait states.  M0 is not saved: no compiler code of these kernels touches it
// (tools/asm_check.py checks the emitted code; M0 is a reserved register, so clang ignores it in a
// clobber list -- "-Winline-asm: reserved registers on the clobber list may not be preserved").  s_add_u32 writes SCC: declared
// clobbered too (without it hipcc kept a comparison in SCC across the statement and the last group's
// surplus-wave selection went wrong -- the rgb bias chunk was never copied).  A surplus wave of the
// last piece (w + WAVES I > NCH - 1) re-copies its previous piece instead: the same bytes to the same
// place.
#ifndef NERF_DMA_LEAN
#define NERF_DMA_LEAN 1
#endif
struct DmaLean {
  const void* gbase;  // packed weights (kernel argument: SGPR pair)
  uint32_t vlane;     // 16 lane + 1024 wave
  uint32_t swave;     // LDS byte address of the ring + 1024 wave (wave-uniform)
  uint32_t wave_u;    // wave (wave-uniform)
};
template <class P, int C0, int NCH, int SLOT_OFF, int I>
__device__ __forceinline__ void fetch_piece_lean(const DmaLean& d) {
  if constexpr (NERF_DIAG_NO_DMA) return;
  constexpr int NU = (NCH + P::WAVES - 1) / P::WAVES;
  constexpr uint32_t GOFF = (uint32_t)(C0 + P::WAVES * I) * 1024u, LOFF = (uint32_t)(SLOT_OFF + P::WAVES * I * 1024);
  static_assert(NCH % P::WAVES == 0 || NU >= 2, "a one-piece group with surplus waves");
  if constexpr (I + 1 < NU || NCH % P::WAVES == 0) {
    const uint32_t voff = d.vlane + GOFF;
    asm volatile("s_add_u32 m0, %1, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %3"
                 :: "v"(voff), "s"(d.swave), "i"(LOFF), "s"(d.gbase) : "memory", "scc");
  } else {
    const uint32_t adj = d.wave_u + P::WAVES * I > (uint32_t)(NCH - 1) ? (uint32_t)P::WAVES * 1024u : 0u;
    const uint32_t voff = d.vlane + (GOFF - adj);
    asm volatile("s_add_u32 m0, %1, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %3"
                 :: "v"(voff), "s"(d.swave - adj), "i"(LOFF), "s"(d.gbase) : "memory", "scc");
  }
}
template <class P, int C0, int NCH, int SLOT_OFF>
__device__ __forceinline__ void fetch_group_lean(const DmaLean& d) {
  constexpr int NU = (NCH + P::WAVES - 1) / P::WAVES;
  sfor<NU>([&](auto ii) { fetch_piece_lean<P, C0, NCH, SLOT_OFF, decltype(ii)::value>(d); });
}

// issue the whole DMA of group G into slot `slot` (group_dma_units pieces per wave)
template <class P, int C0, int NCH, bool LAUNDER = false>
__device__ __forceinline__ void fetch_group(const uint4* gsrc, uint32_t slot_base, int wave, int lane) {
  constexpr int NU = (NCH + P::WAVES - 1) / P::WAVES;
  sfor<NU>([&](auto ii) { fetch_piece<P, C0, NCH, decltype(ii)::value, LAUNDER>(gsrc, slot_base, wave, lane); });
}


// ------------------------------------------------------------------------------------
// positional encoding straight into accumulator-layout tiles
// (freq.py:7-32: [x, sin(2^k x), cos(2^k x)]_k; feature 3 + 6k + {0..2 sin, 3..5 cos})
// ------------------------------------------------------------------------------------
// feature f of an nfreq-band encoding -> (kind, coordinate, band, cos?)
//   kind 0: zero (padding), 1: the raw coordinate, 2: sin/cos(x_dim * 2^k)
struct PeFeat { int kind, dim, k, cos; };
__host__ __device__ constexpr PeFeat pe_feat(int f, int nfreq, int nvalid) {
  if (f >= nvalid) return PeFeat{0, 0, 0, 0};
  if (f < 3) return PeFeat{1, f, 0, 0};
  const int g = f - 3, k = g / 6, r = g % 6;
  if (k >= nfreq) return PeFeat{0, 0, 0, 0};
  return PeFeat{2, r % 3, k, r >= 3 ? 1 : 0};
}

// sin or cos of x * 2^k, three forms (P::PE):
//   PE_FAST (bf16): the angle in revolutions, x * (2^k / 2pi) + (cos ? 1/4 : 0), reduced
//     exactly enough in f64 (|x 2^k| < 2^13 rad keeps ~40 fractional bits), then v_sin_f32 on
//     [0,1) revolutions -- far inside bf16 resolution.
//   PE_LIBM (fp32, the parity path): one libm sincosf of the exact fp32 product x * 2^k (as
//     torch computes x * 2.**k, then sin/cos).  Its large-argument path costs ~140
//     instructions per value, 3-5 % of the fp32 forward, but the cheaper forms below move the
//     4096-ray fine-net L0 gradient 3e-4 from the reference's (a correctly rounded f64 sin
//     does too; libm sincosf: 5e-5, tools/grad_margin.py) against the 1e-4 contract: the fine
//     net's highest PE band amplifies sample-position ulps 512x.
//   PE_POLY (bf16x3, whose own products carry ~1e-5 relative error): the f64 revolution
//     reduction to the nearest quarter turn, t = q/4 + f with |f| <= 1/8, and a Cephes
//     sinf / cosf polynomial of theta = 2 pi f in fp32, chosen and signed by q mod 4:
//     branch-free, ~20 VALU, within 1.6 ulp of sin/cos (forward 12 % faster than libm).
enum PeMode { PE_FAST = 0, PE_LIBM = 1, PE_POLY = 2 };
__device__ __forceinline__ float sin_rev_poly(double t) {
  const double q = __builtin_rint(4.0 * t);
  const double f = __builtin_fma(q, -0.25, t);
  const float th = (float)(f * 6.283185307179586476925286766559);
  const float z = th * th;
  const float s = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z,
                                                -1.6666654611e-1f) * z, th, th);
  const float c = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                                                4.166664568298827e-2f) * z, z, __builtin_fmaf(-0.5f, z, 1.0f));
  const int qi = (int)q;
  const float r = (qi & 1) ? c : s;
  return (qi & 2) ? -r : r;
}

template <int MODE>
__device__ __forceinline__ float pe_trig(float x, double scale_rev, float scale_rad, double phase, bool is_cos) {
  if constexpr (MODE == PE_LIBM) {
    float s, c;
    sincosf(x * scale_rad, &s, &c);
    return is_cos ? c : s;
  } else {
    const double t = __builtin_fma((double)x, scale_rev, phase);
    if constexpr (MODE == PE_FAST) return __builtin_amdgcn_sinf((float)(t - __builtin_floor(t)));
    else return sin_rev_poly(t);
  }
}

// positional encoding straight into accumulator-layout tiles (freq.py:7-32:
// [x, sin(2^k x), cos(2^k x)]_k, feature 3 + 6k + {0..2 sin, 3..5 cos}).  Register rho of
// lane l holds feature 32 tile + acc_row(rho, l >> 5): the two lane halves differ by 4
// features, so each register selects between two compile-time feature descriptors.
template <class P, int TILE, int NFREQ, int NVALID>
__device__ __forceinline__ void pe_tile(typename P::Tile& t, int h, float x0, float x1, float x2) {
  constexpr double INV2PI = 0.15915494309189533576888376337251;
  float vals[16];
  sfor<16>([&](auto rr) {
    constexpr int rho = decltype(rr)::value;
    constexpr PeFeat A = pe_feat(32 * TILE + acc_row(rho, 0), NFREQ, NVALID);
    constexpr PeFeat B = pe_feat(32 * TILE + acc_row(rho, 1), NFREQ, NVALID);
    float v;
    if constexpr (A.kind == 0 && B.kind == 0) {
      v = 0.f;
    } else {
      const int dim = h ? B.dim : A.dim;
      const float x = dim == 0 ? x0 : dim == 1 ? x1 : x2;
      float trig = 0.f;
      if constexpr (A.kind == 2 || B.kind == 2) {
        constexpr int ka = A.kind == 2 ? A.k : (B.kind == 2 ? B.k : 0);
        constexpr int kb = B.kind == 2 ? B.k : ka;
        const int k = h ? kb : ka;
        const bool is_cos = h ? (B.cos != 0) : (A.cos != 0);
        const double srev = INV2PI * (double)(1 << k);
        trig = pe_trig<P::PE>(x, srev, (float)(1 << k), is_cos ? 0.25 : 0.0, is_cos);
      }
      const int kind = h ? B.kind : A.kind;
      v = kind == 2 ? trig : kind == 1 ? x : 0.f;
    }
    if constexpr (P::KIND == K_BF16X3) vals[rho] = v;
    else P::set(t, rho, v);  // (fp32: element-wise keeps the forward's register allocation)
  });
  if constexpr (P::KIND == K_BF16X3) P::pack16(t, vals);
}

// KiB offset of chunk c of tile tau of 32-sample block b in a store of `ntiles` tiles.
// Block-major: one block's tiles are contiguous (a dW job reads a few contiguous runs per
// block instead of one 1-2 KiB piece from each of up to 18 distant tile planes).
__host__ __device__ constexpr int64_t tile_kib(int64_t nblk, int ntiles, int tau, int64_t b, int c, int ch) {
  return (b * ntiles + tau) * ch + c;
}
// KiB stride between consecutive blocks of one tile
__host__ __device__ constexpr int64_t block_stride_kib(int ntiles, int ch) {
  return (int64_t)ntiles * ch;
}

// fragment-native store of one finished tile (mlp_tables.h, "Training stores"): CH
// lane-linear 16-byte stores per lane, each wave-instruction writes 1 KiB contiguous
//
// The training stores (activations, dZ, masks: written once, read once by a later kernel,
// gigabytes per launch) are nontemporal.  Measured per launch at 524,288 samples
// (tools/mlp_bench.py --libs, interleaved): nt takes the training forward 5.22 -> 4.94 ms
// (fp32), 0.737 -> 0.667 (bf16), 2.38 -> 2.02 (bf16x3) and dX 4.49 -> 4.35 / 0.692 -> 0.626 /
// 1.92 -> 1.78 against plain stores; sc1 gained as much on fp32 and less on bf16.
template <int OFF>
__device__ __forceinline__ void store16(uint4* p, uint4 v) {
  if constexpr (NERF_DIAG_NO_STORE) return;
  const u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, (u32x4*)p + OFF / 16);
}
// SCH: chunks stored per tile (P::CH; 2 for a bf16x3 tile stored as its bf16 hi half, the
// bf16 tile-block layout)
template <class P, int SCH = P::CH>
__device__ __forceinline__ void store_tile(void* base, int64_t nblk, int ntiles, int tau, int64_t wblock, int lane,
                                           const typename P::Tile& t) {
  uint4* dst = (uint4*)base + tile_kib(nblk, ntiles, tau, wblock, 0, SCH) * 64 + lane;
  sfor<SCH>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    store16<c * 1024>(dst, P::chunk(t, c));
  });
}


// ReLU masks of the training forward, read by the dX chain: per 32-sample wave block,
// MASK_GROUPS x 64 lanes x 16 B; group l < 8 = layer l's 8 output tiles (tile n -> dword
// n >> 1, bit 8 (n & 1) + mask_bit(rho)), group 8 = the view layer's 4 tiles.  One 16-byte
// store per lane per layer.
__device__ __forceinline__ uint4* mask_slot(void* masks, int64_t wblock, int grp, int lane) {
  return (uint4*)masks + (wblock * MASK_GROUPS + grp) * 64 + lane;
}

// NERF_KEEP_PE_BF3: the bf16x3 forward holds its position-encoding tiles X from L0 to the
// skip input of L5 instead of recomputing them there (its f64-reduced polynomial sin/cos):
// bit-identical, inference forward 1.526 -> 1.498 ms, bf16x3f training forward 1.688 -> 1.668,
// bf16x3 1.872 -> 1.845 at 524,288 samples (r4).  fp32 / bf16 recompute (their register budgets)
#ifndef NERF_KEEP_PE_BF3
#define NERF_KEEP_PE_BF3 1
#endif
template <class P> __host__ __device__ constexpr bool keep_pe() {
  return (P::KIND == K_BF16X3 || P::KIND == K_BF16X3W || P::KIND == K_F32W) && NERF_KEEP_PE_BF3;
}

// ------------------------------------------------------------------------------------
// forward: one wave = 32 samples through all 11 layers; activations stay in registers
// (feature-major accumulator layout = the next layer's B operand).
// ------------------------------------------------------------------------------------
struct FwdArgs {
  const char* wpack;
  const float* pts;          // [M,3]
  const float* dirs;         // [ndir,3] unit view directions
  const int32_t* dir_index;  // [M] or null (then dir = m / samples_per_dir)
  int samples_per_dir;
  int64_t M;
  int64_t nblk;              // 32-sample blocks of the stores (M padded to M_ALIGN) / 32
  float* raw;                // [M,4]
  void* act;                 // [AT_TILES][nblk] tile-blocks or null
  void* masks;               // [nblk][MASK_GROUPS][64] x 16 B or null
  const int32_t* M_dev;      // persistent inference launch: M = min(*M_dev, M_cap), read on the device
  int64_t M_cap;
};

// HALF (bf16x3 only): the training stores keep each tile's bf16 hi half in the bf16 layout
// (2 chunks per tile-block) for a bf16 backward -- the "bf16x3f" tier: bf16x3 outputs, bf16
// gradients.  hi = RNE bf16 of the fp32-class value, exactly what a bf16 forward stores.
template <class P, bool STORE, bool DENSITY, bool PERSIST = false, bool HALF = false>
struct FwdWave {
  using Tile = typename P::Tile;
  static constexpr int CH = P::CH;
  static_assert(!HALF || (P::KIND == K_BF16X3 && STORE), "half stores: bf16x3 training forward only");
  static_assert(finish_schedule_violation<P, 0, DENSITY>() == 0,
                "finish placement (NERF_FINISH_PARTS_* / NERF_FINISH_DELAY) reads a tile pair before its finish part "
                "writes it, or reads a reassigned pend (FinishSchedule)");
  static constexpr int SCH = HALF ? 2 : P::CH;  // chunks stored per tile
  using GT = GroupTable<0, DENSITY, P::CH>;

  const FwdArgs& a;
  const uint4* gw;
  const uint4* lds;
  uint32_t lds_base;
  int lane, wave, h;
  int64_t wblock, m;
  float px, py, pz, dx, dy, dz;
  Tile X[2], D, Ha[8], Hb[8];
  uint32_t mw[4];
  uint32_t one16;   // 0x00010001 in an SGPR, opaque to hipcc (nonzero_bf16x2)
  float alpha, rgb0, rgb1, rgb2;
  lds_cu4* wb;      // current group's slot + 16 h (bias reads)
  uint4 bias[4];
  f32x16 pend;      // finished accumulator awaiting its deferred finish (group_body)
  DmaLean dl;

  __device__ __forceinline__ FwdWave(const FwdArgs& args, const uint4* smem, int64_t blk, int tid)
      : a(args), lds(smem) {
    gw = (const uint4*)a.wpack;
    lds_base = (uint32_t)(uintptr_t)(lds_void*)smem;
    lane = tid & 63;
    wave = tid >> 6;
    h = lane >> 5;
    wblock = blk * P::WAVES + wave;
    m = wblock * 32 + (lane & 31);
    one16 = opaque_one16();
    dl = DmaLean{a.wpack, (uint32_t)(lane * 16 + wave * 1024),
                 (uint32_t)__builtin_amdgcn_readfirstlane(lds_base + (uint32_t)wave * 1024u),
                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)wave)};
  }

  template <int g> __device__ __forceinline__ void fetch() {
    constexpr Group G = GT::t.g[g];
    if constexpr (NERF_DMA_LEAN) fetch_group_lean<P, G.c0, G.nch, (g % NSLOT) * SLOT_CAP * 1024>(dl);
    else fetch_group<P, G.c0, G.nch, PERSIST>(gw, lds_base + (uint32_t)((g % NSLOT) * SLOT_CAP * 1024), wave, lane);
  }
  template <int g, int i> __device__ __forceinline__ void fetch_piece() {
    constexpr Group G = GT::t.g[g];
    if constexpr (NERF_DMA_LEAN) fetch_piece_lean<P, G.c0, G.nch, (g % NSLOT) * SLOT_CAP * 1024, i>(dl);
    else nerf::mlp::fetch_piece<P, G.c0, G.nch, i, PERSIST>(gw, lds_base + (uint32_t)((g % NSLOT) * SLOT_CAP * 1024),
                                                            wave, lane);
  }

  // register tile slot S (TileSlot: Ha/Hb ping-pong, PE tiles X / D); layer L reads
  // slot<fwd_in_slot(L, t)>, its finish writes slot<fwd_out_slot(L, n)>
  template <int S> __device__ __forceinline__ Tile& slot() {
    if constexpr (S >= TS_HA && S < TS_HB) return Ha[S - TS_HA];
    else if constexpr (S >= TS_HB && S < TS_X) return Hb[S - TS_HB];
    else if constexpr (S == TS_X || S == TS_X + 1) return X[S - TS_X];
    else {
      static_assert(S == TS_D, "forward tile slot");
      return D;
    }
  }
  template <int L, int t> __device__ __forceinline__ const Tile& in_tile_L() {
    return slot<fwd_in_slot(L, t)>();
  }

  // vector-memory stores issued by unit u's finish
  static __host__ __device__ constexpr int unit_stores(int u) {
    if (!STORE) return 0;
    const int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
    if (L == LFA) return n < 8 ? SCH : 0;
    if (L == LRGB) return 0;
    return SCH + (n == fwd_out_tiles(L) - 1 ? 1 : 0);  // + the layer's mask store
  }
  static __host__ __device__ constexpr int group_stores(int g) {
    int s = 0;
    for (int u = 0; u < NUNIT_FWD; ++u)
      if (finished_in_group<0, DENSITY, P::CH, cross_finish<P, 0>()>(g, u)) s += unit_stores(u);
    return s;
  }

  // part p of NP of unit (L, n)'s finish: register pairs [8p/NP, 8(p+1)/NP) into the output
  // tile (in place), their mask bits; the last part stores the tile (and the layer's masks)
  template <int L, int n, int p> __device__ __forceinline__ void finish_L_part(const f32x16& acc) {
    constexpr int NP = finish_parts<P>();
    constexpr int K0 = 8 * p / NP, K1 = 8 * (p + 1) / NP;
    constexpr bool LASTP = p == NP - 1;
    if constexpr (L <= L7 || L == LV) {
      Tile& out = slot<fwd_out_slot(L, n)>();
      uint32_t bits = 0;  // this tile's mask bits (mask_bit layout)
      sfor<K1 - K0>([&](auto kk) {
        constexpr int k = K0 + decltype(kk)::value;
        const float a0 = acc[2 * k], a1 = acc[2 * k + 1];
        if constexpr (P::KIND == K_BF16) {
          // bf16: pack the pair first, then ReLU on the packed pair (one VALU for both); the mask
          // bits k / 16 + k from the packed result (as the bf16x3 path, NERF_PACKED_MASK)
          const uint32_t d = relu_bf16x2(pack_bf16(a0, a1));
          if constexpr (STORE && NERF_PACKED_MASK) {
            bits |= nonzero_bf16x2(d, one16) << k;
          } else if constexpr (STORE) {
            bits |= (a0 > 0.f ? 1u : 0u) << mask_bit(2 * k);
            bits |= (a1 > 0.f ? 1u : 0u) << mask_bit(2 * k + 1);
          }
          P::set_dword(out, k, d);
        } else {
          // ReLU as an integer max on the float bits (negative floats are negative ints)
          const int y0 = max(__float_as_int(a0), 0), y1 = max(__float_as_int(a1), 0);
          if constexpr (STORE && P::KIND == K_BF16X3 && NERF_PACKED_MASK) {
            // bit k / 16 + k = the pair's hi halves non-zero: the same bits as y > 0, since RNE keeps
            // every positive fp32 above 2^-134 non-zero in bf16 (pre-activations that small do not occur)
            bits |= nonzero_bf16x2(pack_bf16(__int_as_float(y0), __int_as_float(y1)), one16) << k;
          } else if constexpr (STORE) {
            bits |= min((uint32_t)y0, 1u) << mask_bit(2 * k);
            bits |= min((uint32_t)y1, 1u) << mask_bit(2 * k + 1);
          }
          P::set_pair(out, k, __int_as_float(y0), __int_as_float(y1));
        }
      });
      if constexpr (STORE) {
        if constexpr (K0 == 0 && (n & 1) == 0) mw[n >> 1] = bits;
        else mw[n >> 1] |= bits << (8 * (n & 1));
        if constexpr (LASTP) {
          store_tile<P, SCH>(a.act, a.nblk, AT_TILES, (L == LV ? AT_V : AT_H + 8 * L) + n, wblock, lane, out);
          if constexpr (n == fwd_out_tiles(L) - 1)
            store16<0>(mask_slot(a.masks, wblock, L == LV ? 8 : L, lane),
                       make_uint4(mw[0], mw[1], L == LV ? 0u : mw[2], L == LV ? 0u : mw[3]));
        }
      }
    } else if constexpr (L == LFA) {
      if constexpr (n < 8) {  // feature_linear: no activation
        Tile& out = slot<fwd_out_slot(L, n)>();
        sfor<K1 - K0>([&](auto kk) {
          constexpr int k = K0 + decltype(kk)::value;
          P::set_pair(out, k, acc[2 * k], acc[2 * k + 1]);
        });
        if constexpr (STORE && LASTP) store_tile<P, SCH>(a.act, a.nblk, AT_TILES, AT_F + n, wblock, lane, out);
      } else if constexpr (p == 0) {
        alpha = acc[0];  // alpha_linear: output row 0 = register 0 of lanes 0..31
      }
    } else if constexpr (p == 0) {  // LRGB: rows 0..2 = registers 0..2 of lanes 0..31
      rgb0 = acc[0];
      rgb1 = acc[1];
      rgb2 = acc[2];
    }
  }

  // ---- group_body hooks
  template <int u> static __host__ __device__ constexpr int group_of() {
    int g = 0;
    while (!(GT::t.g[g].u0 <= u && u < GT::t.g[g].u0 + GT::t.g[g].n)) ++g;
    return g;
  }
  template <int u, int t> __device__ __forceinline__ const Tile& in_tile() {
    return in_tile_L<fwd_unit_layer(u), t>();
  }
  // the unit's bias chunk (rows 8q + 4h + {0..3} = lane 2q + h) is the MFMA chain's
  // initial accumulator; it is read one unit ahead
  template <int u> __device__ __forceinline__ void prefetch() {
    constexpr int L = fwd_unit_layer(u);
    constexpr int BOFF = unit_chunk_off<0>(u, CH) - GT::t.g[group_of<u>()].c0 + fwd_in_tiles(L) * CH;
#pragma unroll
    for (int q = 0; q < 4; ++q) bias[q] = as_uint4(wb[BOFF * 64 + 2 * q]);
  }
  template <int u> __device__ __forceinline__ void init(f32x16& acc) {
    constexpr int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
    if constexpr (L == L5 && n == 0 && !keep_pe<P>()) {  // PE recomputed for the skip instead of held through L1..L4
      settle(px);  // opaque to hipcc: it would otherwise CSE this with the L0 tiles and hold them
      settle(py);
      settle(pz);
      pe_tile<P, 0, 10, 63>(X[0], h, px, py, pz);
      pe_tile<P, 1, 10, 63>(X[1], h, px, py, pz);
    }
    if constexpr (L == LV && n == 0) {
      settle(dx);
      settle(dy);
      settle(dz);
      pe_tile<P, 0, 4, 27>(D, h, dx, dy, dz);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc[4 * q + 0] = __uint_as_float(bias[q].x);
      acc[4 * q + 1] = __uint_as_float(bias[q].y);
      acc[4 * q + 2] = __uint_as_float(bias[q].z);
      acc[4 * q + 3] = __uint_as_float(bias[q].w);
    }
  }
  template <int u, int p> __device__ __forceinline__ void finish_part(const f32x16& acc) {
    constexpr int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
    finish_L_part<L, n, p>(acc);
  }

  template <int g> __device__ __forceinline__ void step() {
    constexpr int NG = GT::t.n;
    if constexpr (g + PF < NG && dma_spread<P>() == 0) fetch<g + PF>();
    const uint32_t slot = lds_base + (uint32_t)((g % NSLOT) * SLOT_CAP * 1024);
    wb = lds_ptr(slot + (uint32_t)(h * 16));
    group_body<P, 0, DENSITY, g>(*this, lds_ptr(slot + (uint32_t)(lane * 16)));
    constexpr int N = dma_spread<P>() > 0
        ? handoff_vmcnt_spread<P, 0, DENSITY>(g, [](int u) constexpr { return unit_stores(u); })
        : handoff_vmcnt<P, 0, DENSITY>(g, [](int i) constexpr { return group_stores(i); }, STORE ? 3 * SCH : 0);
    if constexpr (g + 1 < NG) wait_barrier<N>();
  }

  __device__ __forceinline__ void run() {
#if NERF_DIAG_STAMPS
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int64_t ms = m < a.M ? m : a.M - 1;
    px = a.pts[ms * 3 + 0];
    py = a.pts[ms * 3 + 1];
    pz = a.pts[ms * 3 + 2];
    dx = dy = dz = 0.f;
    if constexpr (!DENSITY) {
      const int64_t di = a.dir_index ? (int64_t)a.dir_index[ms] : ms / a.samples_per_dir;
      dx = a.dirs[di * 3 + 0];
      dy = a.dirs[di * 3 + 1];
      dz = a.dirs[di * 3 + 2];
    }
    sfor<(PF < GT::t.n ? PF : GT::t.n)>([&](auto gg) { fetch<decltype(gg)::value>(); });
    pe_tile<P, 0, 10, 63>(X[0], h, px, py, pz);
    pe_tile<P, 1, 10, 63>(X[1], h, px, py, pz);
    if constexpr (STORE) {
      Tile Dt;
      pe_tile<P, 0, 4, 27>(Dt, h, dx, dy, dz);
      store_tile<P, SCH>(a.act, a.nblk, AT_TILES, AT_X, wblock, lane, X[0]);
      store_tile<P, SCH>(a.act, a.nblk, AT_TILES, AT_X + 1, wblock, lane, X[1]);
      store_tile<P, SCH>(a.act, a.nblk, AT_TILES, AT_D, wblock, lane, Dt);
    }
    {  // group 0 landed: younger = the DMAs of groups 1 .. PF - 1 and the PE stores
      constexpr int N0 = [] {
        int n = STORE ? 3 * SCH : 0;
        for (int j = 1; j < PF && j < GT::t.n; ++j) n += group_dma<P, 0, DENSITY>(j);
        return n;
      }();
      wait_barrier<N0>();
    }
#if NERF_DIAG_STAMPS
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
#endif
    settle(dx);
    settle(dy);
    settle(dz);
    sfor<GT::t.n>([&](auto gg) { step<decltype(gg)::value>(); });
    if (h == 0 && m < a.M)
      *(float4*)(a.raw + m * 4) = DENSITY ? make_float4(0.f, 0.f, 0.f, alpha) : make_float4(rgb0, rgb1, rgb2, alpha);
#if NERF_DIAG_STAMPS
    // (diagnostic only) wave 0 lane 0 of each workgroup overwrites raw rows 0-1 of its block:
    // hw id, xcc id, entry / prologue-done / end (s_memrealtime)
    const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
    if (wave == 0 && lane == 0) {
      uint32_t* d = (uint32_t*)(a.raw + (wblock * 32) * 4);
      d[0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      d[1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
      d[2] = (uint32_t)t0, d[3] = (uint32_t)(t0 >> 32);
      d[4] = (uint32_t)t1, d[5] = (uint32_t)(t1 >> 32);
      d[6] = (uint32_t)t2, d[7] = (uint32_t)(t2 >> 32);
    }
#endif
  }
};

// ------------------------------------------------------------------------------------
// The wide bf16x3 forward (round 6, PBF3W): one wave = 16 samples on v_mfma_f32_16x16x32_bf16, 8 waves
// per workgroup, two per SIMD.  The bf16x3 forward of the 32x32 kernels above holds 32 samples' hi / lo
// activation tiles per wave in ~370 registers -- one wave per SIMD, so nothing feeds the matrix pipe
// while a wave runs its epilogue (ReLU, hi / lo split, masks, stores) or waits on LDS; with 16 samples
// a wave needs ~200 registers and the two waves of a SIMD overlap each other's epilogues and waits.
// Same weight ring (2 x 72 KiB LDS slots, LDS-DMA one group ahead, counted hand-offs) and group
// pipeline (group_body, finish parts, spread DMA) over 16-row units (DIR 2).
//
// Training stores go to the 32x32 fragment layout the dX / dW kernels read (mlp_tables.h "Training
// stores"): a 32-sample tile-block spans the two waves of a SIMD pair (wave & 1 = its half of the
// samples) and two 16-row output tiles (old chunk c = tile m & 1).  Old lane L = sample (L & 31) + 32 h
// holds features 16 c + 4 h + {0..3} then 16 c + 8 + 4 h + {0..3}: exactly the 4 rows of this kernel's
// lane (s, g = h) and of lane (s, g = h + 2) -- so every lane writes its 8 bytes (4 bf16) with one
// global_store_dwordx2 at 16 L + 8 (g >> 1), no exchange.  The ReLU-mask bits of old lane L come from the
// lanes l and l + 32 of one wave: combined with one v_permlane32_swap per mask dword at the layer's end.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void store8(char* p, uint32_t lo, uint32_t hi) {
  if constexpr (NERF_DIAG_NO_STORE) return;
  typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store((u32x2v){lo, hi}, (u32x2v*)p);  // (plain stores measured: 1.536 -> 1.561 ms, r6)
}
__device__ __forceinline__ uint32_t get_dword(const bf16x8& v, int k) {
  const uint4 u = __builtin_bit_cast(uint4, v);
  return k == 0 ? u.x : k == 1 ? u.y : k == 2 ? u.z : u.w;
}
__device__ __forceinline__ void set_dword8(bf16x8& v, int k, uint32_t d) {
  uint4 u = __builtin_bit_cast(uint4, v);
  if (k == 0) u.x = d;
  else if (k == 1) u.y = d;
  else if (k == 2) u.z = d;
  else u.w = d;
  v = __builtin_bit_cast(bf16x8, u);
}
// position encoding of K-block TILE in the PBF3W B-operand layout: element e of lane group g is feature
// 32 TILE + k16_feat(g, e); the same fp32 values as pe_tile<PBF3> (PE_POLY), split hi / lo
template <class T> __device__ __forceinline__ T sel4(int g, T a0, T a1, T a2, T a3) {
  return (g & 2) ? ((g & 1) ? a3 : a2) : ((g & 1) ? a1 : a0);  // (branch-free selects on the lane group)
}
template <class P, int TILE, int NFREQ, int NVALID>
__device__ __forceinline__ void pe_kblock(typename P::Tile& t, int g, float x0, float x1, float x2) {
  constexpr double INV2PI = 0.15915494309189533576888376337251;
  float v[8];
  sfor<8>([&](auto ee) {
    constexpr int e = decltype(ee)::value;
    constexpr PeFeat F0 = pe_feat(32 * TILE + k16_feat(0, e), NFREQ, NVALID);
    constexpr PeFeat F1 = pe_feat(32 * TILE + k16_feat(1, e), NFREQ, NVALID);
    constexpr PeFeat F2 = pe_feat(32 * TILE + k16_feat(2, e), NFREQ, NVALID);
    constexpr PeFeat F3 = pe_feat(32 * TILE + k16_feat(3, e), NFREQ, NVALID);
    // every candidate is chosen at compile time; only the lane group selects among them
    const float c0 = F0.dim == 0 ? x0 : F0.dim == 1 ? x1 : x2, c1 = F1.dim == 0 ? x0 : F1.dim == 1 ? x1 : x2;
    const float c2 = F2.dim == 0 ? x0 : F2.dim == 1 ? x1 : x2, c3 = F3.dim == 0 ? x0 : F3.dim == 1 ? x1 : x2;
    const float x = sel4(g, c0, c1, c2, c3);
    float trig = 0.f;
    if constexpr (F0.kind == 2 || F1.kind == 2 || F2.kind == 2 || F3.kind == 2) {
      if constexpr (P::PE == PE_LIBM) {  // (PF32W: sincosf of the exact fp32 x * 2^k, as PF32's pe_tile)
        const float srad = sel4(g, (float)(1 << F0.k), (float)(1 << F1.k), (float)(1 << F2.k), (float)(1 << F3.k));
        const bool is_cos = sel4(g, F0.cos != 0, F1.cos != 0, F2.cos != 0, F3.cos != 0);
        trig = pe_trig<PE_LIBM>(x, 0.0, srad, 0.0, is_cos);
      } else {
        const double srev = sel4(g, INV2PI * (double)(1 << F0.k), INV2PI * (double)(1 << F1.k),
                                 INV2PI * (double)(1 << F2.k), INV2PI * (double)(1 << F3.k));
        const double ph = sel4(g, F0.cos ? 0.25 : 0.0, F1.cos ? 0.25 : 0.0, F2.cos ? 0.25 : 0.0, F3.cos ? 0.25 : 0.0);
        trig = pe_trig<PE_POLY>(x, srev, 0.f, ph, false);
      }
    }
    v[e] = sel4(g, F0.kind == 2 ? trig : F0.kind == 1 ? x : 0.f, F1.kind == 2 ? trig : F1.kind == 1 ? x : 0.f,
                F2.kind == 2 ? trig : F2.kind == 1 ? x : 0.f, F3.kind == 2 ? trig : F3.kind == 1 ? x : 0.f);
  });
  if constexpr (P::KIND == K_F32W) {
#pragma unroll
    for (int e = 0; e < 8; ++e) t.v[e] = v[e];
  } else {
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hw[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
      lw[k] = pack_bf16(v[2 * k] - __uint_as_float(hw[k] << 16), v[2 * k + 1] - __uint_as_float(hw[k] & 0xffff0000u));
    }
    t.hi = __builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
    t.lo = __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
  }
}

template <class P, bool STORE, bool DENSITY, bool PERSIST = false, bool HALF = false>
struct FwdWave16 {
  using Tile = typename P::Tile;
  using Acc = f32x4;
  static constexpr bool F32 = P::KIND == K_F32W;
  static_assert(wide_kind<P>() && (!HALF || (!F32 && STORE)), "FwdWave16: PBF3W (HALF: bf16x3f stores) or PF32W");
  static_assert(!F32 || (STORE && !PERSIST), "PF32W: the training forward only");
  static constexpr int CH = P::CH;
  static constexpr int SCH = HALF ? 2 : 4;  // chunks of a stored tile-block: bf16 hi (bf16x3f), hi + lo, or fp32
  // stores per output tile: PBF3W one 8-byte store per half (hi [+ lo]); PF32W one 16-byte store
  static constexpr int SST = F32 ? 1 : HALF ? 1 : 2;
  // (r6, measured and removed: the two 16-row tiles of one old tile stored together, one 16-byte store per lane
  // with the halves exchanged by v_permlane32_swap -- bit-identical, bf16x3f training forward 1.502 -> 1.573 ms,
  // bf16x3 1.660 -> 1.769; profiles/r6/pair_store_ab.json)
  static constexpr int PRO_ST = NERF_DIAG_NO_ACT ? 0 : 6 * SST;  // the prologue's PE stores (3 K-blocks x 2 halves)
  using GT = GroupTable<2, DENSITY, P::CH>;
  static_assert(finish_schedule_violation<P, 2, DENSITY>() == 0,
                "finish placement (NERF_FINISH_PARTS_* / NERF_FINISH_DELAY) reads a tile pair before its finish part "
                "writes it, or reads a reassigned pend (FinishSchedule)");

  const FwdArgs& a;
  uint32_t lds_base;
  int lane, wave, s, g;
  int64_t m;        // this lane's sample
  int64_t wb32;     // the 32-sample block of the training stores
  uint32_t st_off;  // byte offset of this lane's 8 bytes in a 1-KiB chunk of the stores (PF32W: its 16 bytes,
                    // + 1 KiB (g >> 1): chunk 2 (mt & 1) + (g >> 1) of the fp32 tile-block)
  uint32_t lold;    // old-layout lane of the mask store: sample (16 (wave & 1) + s) + 32 (g & 1)
  uint32_t gsh;     // 2 (g >> 1): offset of this lane's mask bits among an old register pair group
  float px, py, pz, dx, dy, dz;
  Tile X[2], D, Ha[8], Hb[8];
  uint32_t mw[4];
  uint32_t one16;
  float alpha, rgb0, rgb1, rgb2;
  lds_cu4* wbg;     // current group's slot + 16 g (bias reads)
  uint4 bias;
  Acc pend;
  DmaLean dl;

  __device__ __forceinline__ FwdWave16(const FwdArgs& args, const uint4* smem, int64_t blk, int tid) : a(args) {
    lds_base = (uint32_t)(uintptr_t)(lds_void*)smem;
    lane = tid & 63;
    wave = tid >> 6;
    s = lane & 15;
    g = lane >> 4;
    m = (blk * P::WAVES + wave) * 16 + s;
    wb32 = blk * (P::WAVES / 2) + (wave >> 1);
    const uint32_t sb = 16u * (uint32_t)(wave & 1) + (uint32_t)s;
    lold = sb + 32u * (uint32_t)(g & 1);
    st_off = 16u * lold + (F32 ? 1024u : 8u) * (uint32_t)(g >> 1);
    gsh = 2u * (uint32_t)(g >> 1);
    one16 = opaque_one16();
    dl = DmaLean{a.wpack, (uint32_t)(lane * 16 + wave * 1024),
                 (uint32_t)__builtin_amdgcn_readfirstlane(lds_base + (uint32_t)wave * 1024u),
                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)wave)};
  }

  template <int gi> __device__ __forceinline__ void fetch() {
    constexpr Group G = GT::t.g[gi];
    fetch_group_lean<P, G.c0, G.nch, (gi % NSLOT) * SLOT_CAP * 1024>(dl);
  }
  template <int gi, int i> __device__ __forceinline__ void fetch_piece() {
    constexpr Group G = GT::t.g[gi];
    fetch_piece_lean<P, G.c0, G.nch, (gi % NSLOT) * SLOT_CAP * 1024, i>(dl);
  }
  template <int S> __device__ __forceinline__ Tile& slot() {
    if constexpr (S >= TS_HA && S < TS_HB) return Ha[S - TS_HA];
    else if constexpr (S >= TS_HB && S < TS_X) return Hb[S - TS_HB];
    else if constexpr (S == TS_X || S == TS_X + 1) return X[S - TS_X];
    else {
      static_assert(S == TS_D, "forward tile slot");
      return D;
    }
  }
  template <int u> static __host__ __device__ constexpr int layer_of() { return fwd16_unit_layer(u); }
  template <int u> static __host__ __device__ constexpr int tile_of() { return u - fwd16_unit_first(fwd16_unit_layer(u)); }

  // vector-memory stores issued by unit u's finish
  static __host__ __device__ constexpr int unit_stores(int u) {
    if (!STORE) return 0;
    const int L = fwd16_unit_layer(u), mt = u - fwd16_unit_first(L);
    constexpr int ST = NERF_DIAG_NO_ACT ? 0 : SST, MS = NERF_DIAG_NO_MASK ? 0 : 1;
    if (L == LFA) return mt < 16 ? ST : 0;
    if (L == LRGB) return 0;
    return ST + (mt == fwd16_out_tiles(L) - 1 ? MS : 0);  // + the layer's mask store
  }
  static __host__ __device__ constexpr int group_stores(int gi) {
    int n = 0;
    for (int u = 0; u < NUNIT_FWD16; ++u)
      if (finished_in_group<2, DENSITY, P::CH, cross_finish<P, 2>()>(gi, u)) n += unit_stores(u);
    return n;
  }
  // the training stores of one 32-feature tile (a K-block, or the two 16-row tiles that fill it): old
  // tile tau, 8 bytes of chunk c (hi) [and c + 2 (lo)] at this lane's slot
  __device__ __forceinline__ void store_half(int tau, int c, uint32_t h0, uint32_t h1, uint32_t l0, uint32_t l1) {
    if constexpr (NERF_DIAG_NO_ACT) return;
    char* base = (char*)a.act + (((wb32 * AT_TILES + tau) * SCH + c) << 10) + st_off;
    store8(base, h0, h1);
    if constexpr (!HALF) store8(base + 2048, l0, l1);
  }
  // PF32W: output-tile half hf of fp32 tile tau (values v[4 hf .. 4 hf + 3]) = old lane lold's 16 bytes of chunk
  // 2 hf + (g >> 1) (old register rho = 4 (2 hf + (g >> 1)) + e holds feature 16 hf + 4 g + e, acc_row)
  __device__ __forceinline__ void store_f32(int tau, int hf, const Tile& t) {
    if constexpr (NERF_DIAG_NO_ACT) return;
    char* base = (char*)a.act + (((wb32 * AT_TILES + tau) * SCH + 2 * hf) << 10) + st_off;
    store16<0>((uint4*)base, make_uint4(__float_as_uint(t.v[4 * hf]), __float_as_uint(t.v[4 * hf + 1]),
                                        __float_as_uint(t.v[4 * hf + 2]), __float_as_uint(t.v[4 * hf + 3])));
  }
  __device__ __forceinline__ void store_kblock(int tau, const Tile& t) {
    if constexpr (F32) {
      store_f32(tau, 0, t);
      store_f32(tau, 1, t);
    } else {
      store_half(tau, 0, get_dword(t.hi, 0), get_dword(t.hi, 1), get_dword(t.lo, 0), get_dword(t.lo, 1));
      store_half(tau, 1, get_dword(t.hi, 2), get_dword(t.hi, 3), get_dword(t.lo, 2), get_dword(t.lo, 3));
    }
  }

  // ---- group_body hooks
  template <int u> static __host__ __device__ constexpr int group_of() {
    int gi = 0;
    while (!(GT::t.g[gi].u0 <= u && u < GT::t.g[gi].u0 + GT::t.g[gi].n)) ++gi;
    return gi;
  }
  template <int u, int t> __device__ __forceinline__ const Tile& in_tile() {
    return slot<fwd_in_slot(layer_of<u>(), t)>();
  }
  // the unit's bias chunk (rows 4 g + {0..3} = lane g) is the MFMA chain's initial accumulator, read one unit ahead
  template <int u> __device__ __forceinline__ void prefetch() {
    constexpr int BOFF = unit_chunk_off<2>(u, CH) - GT::t.g[group_of<u>()].c0 + fwd_in_tiles(layer_of<u>()) * CH;
    bias = as_uint4(wbg[BOFF * 64]);
  }
  template <int u> __device__ __forceinline__ void init(Acc& acc) {
    constexpr int L = layer_of<u>(), mt = tile_of<u>();
    if constexpr (L == L5 && mt == 0 && !keep_pe<P>()) {
      settle(px);
      settle(py);
      settle(pz);
      pe_kblock<P, 0, 10, 63>(X[0], g, px, py, pz);
      pe_kblock<P, 1, 10, 63>(X[1], g, px, py, pz);
    }
    if constexpr (L == LV && mt == 0) {
      settle(dx);
      settle(dy);
      settle(dz);
      pe_kblock<P, 0, 4, 27>(D, g, dx, dy, dz);
    }
    acc[0] = __uint_as_float(bias.x);
    acc[1] = __uint_as_float(bias.y);
    acc[2] = __uint_as_float(bias.z);
    acc[3] = __uint_as_float(bias.w);
  }
  // part p of NP of output tile mt's finish: its register pairs [2p/NP, 2(p+1)/NP) into half mt & 1 of the
  // output K-block (in place), their mask bits; the last part stores (and the layer's last tile the masks)
  template <int u, int p> __device__ __forceinline__ void finish_part(const Acc& acc) {
    constexpr int L = layer_of<u>(), mt = tile_of<u>();
    constexpr int NP = finish_parts<P>();
    constexpr int K0 = 2 * p / NP, K1 = 2 * (p + 1) / NP;
    constexpr bool LASTP = p == NP - 1;
    if constexpr (L <= L7 || L == LV || (L == LFA && mt < 16)) {
      constexpr bool RELU = L != LFA;  // feature_linear: no activation
      constexpr int Q = 2 * (mt & 1);   // the K-block dwords of this tile: Q, Q + 1
      Tile& out = slot<fwd_out_slot(L, mt >> 1)>();
      uint32_t bits = 0;
      sfor<K1 - K0>([&](auto kk) {
        constexpr int k = K0 + decltype(kk)::value;
        float y0 = acc[2 * k], y1 = acc[2 * k + 1];
        if constexpr (RELU) {
          y0 = __int_as_float(max(__float_as_int(y0), 0));
          y1 = __int_as_float(max(__float_as_int(y1), 0));
        }
        if constexpr (F32) {
          // bits k / 16 + k: the pair's values non-zero (after the ReLU: > 0), the bf16 path's bit layout
          if constexpr (STORE && RELU && !NERF_DIAG_NO_MASK)
            bits |= (min((uint32_t)__float_as_int(y0), 1u) | (min((uint32_t)__float_as_int(y1), 1u) << 16)) << k;
          out.v[2 * Q + 2 * k] = y0;
          out.v[2 * Q + 2 * k + 1] = y1;
        } else {
          const uint32_t hw = pack_bf16(y0, y1);
          const uint32_t lw = pack_bf16(y0 - __uint_as_float(hw << 16), y1 - __uint_as_float(hw & 0xffff0000u));
          if constexpr (STORE && RELU && !NERF_DIAG_NO_MASK) bits |= nonzero_bf16x2(hw, one16) << k;  // (as PBF3)
          set_dword8(out.hi, Q + k, hw);
          set_dword8(out.lo, Q + k, lw);
        }
      });
      if constexpr (STORE) {
        constexpr int n = mt >> 1, d = mt >> 2;  // old 32-row tile, its mask dword
        if constexpr (RELU && !NERF_DIAG_NO_MASK) {
          // value 2k + j of this lane = old register rho = 4 (2 (mt & 1) + (g >> 1)) + 2k + j of old tile n, old
          // lane half h = g & 1: mask bit 8 (n & 1) + (rho >> 1) + 16 (rho & 1) = [bit k / 16 + k] << (C + gsh)
          constexpr uint32_t C = 8 * (n & 1) + 4 * (mt & 1);
          const uint32_t b = bits << (C + gsh);
          if constexpr ((mt & 3) == 0 && p == 0) mw[d] = b;
          else mw[d] |= b;
        }
        if constexpr (LASTP) {
          constexpr int tau = (L == LV ? AT_V : L == LFA ? AT_F : AT_H + 8 * L) + n;
          if constexpr (F32) store_f32(tau, mt & 1, out);
          else store_half(tau, mt & 1, get_dword(out.hi, Q), get_dword(out.hi, Q + 1), get_dword(out.lo, Q),
                          get_dword(out.lo, Q + 1));
          if constexpr (RELU && !NERF_DIAG_NO_MASK && mt == fwd16_out_tiles(L) - 1) {
            // old lane L gets its bits from lanes l and l + 32 (g = h, h + 2): OR in the partner's dwords; lanes l
            // and l + 32 then hold the same 16 bytes for the same old lane and both store them
            constexpr int ND = L == LV ? 2 : 4;
            uint32_t full[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int q = 0; q < ND; ++q) {
              const auto r = __builtin_amdgcn_permlane32_swap(mw[q], mw[q], false, false);
              full[q] = mw[q] | (lane < 32 ? r[1] : r[0]);
            }
            store16<0>((uint4*)((char*)a.masks + ((wb32 * MASK_GROUPS + (L == LV ? 8 : L)) * 64 + lold) * 16),
                       make_uint4(full[0], full[1], full[2], full[3]));
          }
        }
      }
    } else if constexpr (L == LFA) {  // the alpha row: row 0 = register 0 of lane group 0
      if constexpr (p == 0) alpha = acc[0];
    } else if constexpr (p == 0) {    // LRGB: rows 0..2 = registers 0..2 of lane group 0
      rgb0 = acc[0];
      rgb1 = acc[1];
      rgb2 = acc[2];
    }
  }

  template <int gi> __device__ __forceinline__ void step() {
    constexpr int NG = GT::t.n;
    if constexpr (gi + PF < NG && dma_spread<P>() == 0) fetch<gi + PF>();
    const uint32_t sl = lds_base + (uint32_t)((gi % NSLOT) * SLOT_CAP * 1024);
    wbg = lds_ptr(sl + (uint32_t)(g * 16));
    group_body<P, 2, DENSITY, gi>(*this, lds_ptr(sl + (uint32_t)(lane * 16)));
    constexpr int N = dma_spread<P>() > 0
        ? handoff_vmcnt_spread<P, 2, DENSITY>(gi, [](int u) constexpr { return unit_stores(u); })
        : handoff_vmcnt<P, 2, DENSITY>(gi, [](int i) constexpr { return group_stores(i); }, STORE ? PRO_ST : 0);
    if constexpr (gi + 1 < NG) wait_barrier<N>();
  }

  __device__ __forceinline__ void run() {
    const int64_t ms = m < a.M ? m : a.M - 1;
    px = a.pts[ms * 3 + 0];
    py = a.pts[ms * 3 + 1];
    pz = a.pts[ms * 3 + 2];
    dx = dy = dz = 0.f;
    if constexpr (!DENSITY) {
      const int64_t di = a.dir_index ? (int64_t)a.dir_index[ms] : ms / a.samples_per_dir;
      dx = a.dirs[di * 3 + 0];
      dy = a.dirs[di * 3 + 1];
      dz = a.dirs[di * 3 + 2];
    }
    sfor<(PF < GT::t.n ? PF : GT::t.n)>([&](auto gg) { fetch<decltype(gg)::value>(); });
    pe_kblock<P, 0, 10, 63>(X[0], g, px, py, pz);
    pe_kblock<P, 1, 10, 63>(X[1], g, px, py, pz);
    if constexpr (STORE) {
      Tile Dt;
      pe_kblock<P, 0, 4, 27>(Dt, g, dx, dy, dz);
      store_kblock(AT_X, X[0]);
      store_kblock(AT_X + 1, X[1]);
      store_kblock(AT_D, Dt);
    }
    {  // group 0 landed: younger = the DMAs of groups 1 .. PF - 1 and the PE stores (3 K-blocks x 2 halves)
      constexpr int N0 = [] {
        int n = STORE ? PRO_ST : 0;
        for (int j = 1; j < PF && j < GT::t.n; ++j) n += group_dma<P, 2, DENSITY>(j);
        return n;
      }();
      wait_barrier<N0>();
    }
    settle(dx);
    settle(dy);
    settle(dz);
    sfor<GT::t.n>([&](auto gg) { step<decltype(gg)::value>(); });
    if (g == 0 && m < a.M)
      *(float4*)(a.raw + m * 4) = DENSITY ? make_float4(0.f, 0.f, 0.f, alpha) : make_float4(rgb0, rgb1, rgb2, alpha);
  }
};

template <class P, bool STORE, bool DENSITY, bool PERSIST, bool HALF>
using FwdWaveOf = std::conditional_t<wide_kind<P>(), FwdWave16<P, STORE, DENSITY, PERSIST, HALF>,
                                     FwdWave<P, STORE, DENSITY, PERSIST, HALF>>;

// PERSIST (inference only): the sample count is read on the device (a.M_dev, e.g. the grid
// march's gather count: no host round trip sizes the launch) and a grid of one wave of
// workgroups loops over the sample blocks; the barrier at the end of each block keeps the next
// block's prologue DMA out of the ring slot still being read.
template <class P, bool STORE, bool DENSITY, bool PERSIST, bool HALF = false>
__global__ void __launch_bounds__(P::WAVES * 64) fwd_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem_u4[];
  if constexpr (!PERSIST) {
    FwdWaveOf<P, STORE, DENSITY, false, HALF> w(a, smem_u4, blockIdx.x, threadIdx.x);
    w.run();
  } else {
    static_assert(!STORE, "the persistent forward is inference only");
    const int64_t cnt = a.M_dev[0];
    FwdArgs b = a;
    b.M = cnt < a.M_cap ? cnt : a.M_cap;
    for (int64_t blk = blockIdx.x; blk * samples_per_block<P>() < b.M; blk += gridDim.x) {
      // the thread id, laundered per block: every lane-dependent address (the weight DMA sources,
      // the LDS read bases) is then recomputed inside the body, as in the one-block kernel,
      // instead of being hoisted out of the loop and held in registers across it (spills)
      int tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      FwdWaveOf<P, STORE, DENSITY, true, false> w(b, smem_u4, blk, tid);
      w.run();
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------------------------------
// backward dX chain: W^T products + ReLU masks, 32 samples per wave, storing every
// layer's output gradient (pre-activation dZ) fragment-native for the dW GEMMs.
// Stages (mlp_tables.h BStage): bRGB -> dZv, bV -> dfeature, bFA -> dZ7, b7..b1 -> dZ6..dZ0.
// ------------------------------------------------------------------------------------
// (dz tile, mask group or -1) of output tile j of dX stage s
__host__ __device__ constexpr int bwd_dz_tile(int s, int j) {
  return s == B_RGB ? ZT_V + j : s == B_V ? ZT_F + j : s == B_FA ? ZT_H + 56 + j : ZT_H + 8 * (bwd_fwd_layer(s) - 1) + j;
}
__host__ __device__ constexpr int bwd_mask_group(int s) {
  return s == B_RGB ? 8 : s == B_V ? -1 : s == B_FA ? 7 : bwd_fwd_layer(s) - 1;
}

struct DxArgs {
  const char* wpack_t;  // W^T chunks
  const float* d_raw;   // [M,4]
  int64_t M, nblk;
  const void* masks;    // [nblk][MASK_GROUPS][64] x 16 B
  void* dz;             // [ZT_TILES][nblk] tile-blocks
};

template <class P>
struct DxWave {
  using Tile = typename P::Tile;
  static constexpr int CH = P::CH;
  using GT = GroupTable<1, false, P::CH>;
  static_assert(finish_schedule_violation<P, 1, false>() == 0,
                "finish placement (NERF_FINISH_PARTS_* / NERF_FINISH_DELAY) reads a tile pair before its finish part "
                "writes it, or reads a reassigned pend (FinishSchedule)");

  const DxArgs& a;
  const uint4* gw;
  const uint4* lds;
  uint32_t lds_base;
  int lane, wave, h;
  int64_t wblock, m;
  Tile G, DA, Ha[8], Hb[8];
  uint4 mk[MASK_GROUPS];
  f32x16 pend;      // finished accumulator awaiting its deferred finish (group_body)
  DmaLean dl;

  __device__ __forceinline__ DxWave(const DxArgs& args, const uint4* smem) : a(args), lds(smem) {
    gw = (const uint4*)a.wpack_t;
    lds_base = (uint32_t)(uintptr_t)(lds_void*)smem;
    lane = threadIdx.x & 63;
    wave = threadIdx.x >> 6;
    h = lane >> 5;
    wblock = (int64_t)blockIdx.x * P::WAVES + wave;
    m = wblock * 32 + (lane & 31);
    dl = DmaLean{a.wpack_t, (uint32_t)(lane * 16 + wave * 1024),
                 (uint32_t)__builtin_amdgcn_readfirstlane(lds_base + (uint32_t)wave * 1024u),
                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)wave)};
  }

  template <int g> __device__ __forceinline__ void fetch() {
    constexpr Group Gr = GT::t.g[g];
    if constexpr (NERF_DMA_LEAN) fetch_group_lean<P, Gr.c0, Gr.nch, (g % NSLOT) * SLOT_CAP * 1024>(dl);
    else fetch_group<P, Gr.c0, Gr.nch>(gw, lds_base + (uint32_t)((g % NSLOT) * SLOT_CAP * 1024), wave, lane);
  }
  template <int g, int i> __device__ __forceinline__ void fetch_piece() {
    constexpr Group Gr = GT::t.g[g];
    if constexpr (NERF_DMA_LEAN) fetch_piece_lean<P, Gr.c0, Gr.nch, (g % NSLOT) * SLOT_CAP * 1024, i>(dl);
    else nerf::mlp::fetch_piece<P, Gr.c0, Gr.nch, i>(gw, lds_base + (uint32_t)((g % NSLOT) * SLOT_CAP * 1024), wave,
                                                     lane);
  }
  static __host__ __device__ constexpr int unit_stores(int) { return CH; }

  // register tile slot S (TileSlot: Ha/Hb ping-pong, seeds G / DA); stage s reads
  // slot<bwd_in_slot(s, t)>, its finish writes slot<bwd_out_slot(s, j)>
  template <int S> __device__ __forceinline__ Tile& slot() {
    if constexpr (S >= TS_HA && S < TS_HB) return Ha[S - TS_HA];
    else if constexpr (S >= TS_HB && S < TS_X) return Hb[S - TS_HB];
    else if constexpr (S == TS_G) return G;
    else {
      static_assert(S == TS_DA, "dX tile slot");
      return DA;
    }
  }
  template <int s, int t> __device__ __forceinline__ const Tile& in_tile_S() { return slot<bwd_in_slot(s, t)>(); }
  static __host__ __device__ constexpr int dz_tile(int s, int j) { return bwd_dz_tile(s, j); }
  static __host__ __device__ constexpr int mask_group(int s) { return bwd_mask_group(s); }
  static __host__ __device__ constexpr int group_stores(int g) {
    int s = 0;
    for (int u = 0; u < NUNIT_BWD; ++u)
      if (finished_in_group<1, false, P::CH, cross_finish<P, 1>()>(g, u)) s += CH;
    return s;
  }

  // ---- group_body hooks
  template <int u, int t> __device__ __forceinline__ const Tile& in_tile() {
    return in_tile_S<bwd_unit_stage(u), t>();
  }
  template <int u> __device__ __forceinline__ void prefetch() {}
  template <int u> __device__ __forceinline__ void init(f32x16& acc) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  }
  // part p of NP of unit u's finish: register pairs [8p/NP, 8(p+1)/NP) masked by the forward's
  // ReLU bits into the output-gradient tile (in place); the last part stores the tile
  template <int u, int p> __device__ __forceinline__ void finish_part(const f32x16& acc) {
    constexpr int s = bwd_unit_stage(u), j = u - bwd_unit_first(s);
    constexpr int mg = mask_group(s);
    constexpr int NP = finish_parts<P>();
    constexpr int K0 = 8 * p / NP, K1 = 8 * (p + 1) / NP;
    uint32_t w = 0xFFFFFFFFu;  // this tile's bits at mask_bit(rho) (bf16: + 8 for an odd tile)
    if constexpr (mg >= 0) {
      w = (j >> 1) == 0 ? mk[mg].x : (j >> 1) == 1 ? mk[mg].y : (j >> 1) == 2 ? mk[mg].z : mk[mg].w;
      if constexpr (P::KIND != K_BF16) w >>= 8 * (j & 1);
    }
    // bf16: bits b, 16 + b of pair k (b = k + 8 (j & 1)) -> 0xFFFF / 0 halves: each 16-bit half shifted
    // so its bit lands on bit 15, then arithmetic-shifted back (v_pk_lshlrev_b16 + v_pk_ashrrev_i16;
    // was shift, and, v_mul_u32_u24: 2,614 VALU instead of 3,158 in the dX, 0.591 -> 0.587 ms, r5)
    auto half_mask = [&](auto kk) {
      constexpr unsigned short SH = 15 - decltype(kk)::value - 8 * (j & 1);
      const u16x2 t = __builtin_bit_cast(u16x2, w) << (u16x2){SH, SH};
      return __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2, t) >> (i16x2){15, 15});
    };
    Tile& out = slot<bwd_out_slot(s, j)>();
    sfor<K1 - K0>([&](auto kk) {
      constexpr int k = K0 + decltype(kk)::value;
      if constexpr (P::KIND == K_BF16) {
        uint32_t d = pack_bf16(acc[2 * k], acc[2 * k + 1]);
        if constexpr (mg >= 0) d &= half_mask(std::integral_constant<int, k>{});
        P::set_dword(out, k, d);
      } else {  // (bf16x3: the same half masks on the split hi / lo pairs measured 1.3 % slower, r5)
        const float y0 = ((w >> mask_bit(2 * k)) & 1u) ? acc[2 * k] : 0.f;
        const float y1 = ((w >> mask_bit(2 * k + 1)) & 1u) ? acc[2 * k + 1] : 0.f;
        P::set_pair(out, k, y0, y1);
      }
    });
    if constexpr (p == NP - 1) store_tile<P>(a.dz, a.nblk, ZT_TILES, dz_tile(s, j), wblock, lane, out);
  }

  template <int g> __device__ __forceinline__ void step() {
    constexpr int NG = GT::t.n;
    if constexpr (g + PF < NG && dma_spread<P>() == 0) fetch<g + PF>();
    const uint32_t slot = lds_base + (uint32_t)((g % NSLOT) * SLOT_CAP * 1024);
    group_body<P, 1, false, g>(*this, lds_ptr(slot + (uint32_t)(lane * 16)));
    constexpr int N = dma_spread<P>() > 0
        ? handoff_vmcnt_spread<P, 1, false>(g, [](int u) constexpr { return unit_stores(u); })
        : handoff_vmcnt<P, 1, false>(g, [](int i) constexpr { return group_stores(i); }, 2 * CH);
    if constexpr (g + 1 < NG) wait_barrier<N>();
  }

  __device__ __forceinline__ void run() {
    // output gradients of rgb_linear (rows 0..2) and alpha_linear (row 0): lanes 0..31
    const float4 gr = m < a.M ? *(const float4*)(a.d_raw + m * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < MASK_GROUPS; ++i) mk[i] = *mask_slot((void*)a.masks, wblock, i, lane);
    sfor<(PF < GT::t.n ? PF : GT::t.n)>([&](auto gg) { fetch<decltype(gg)::value>(); });
#pragma unroll
    for (int rho = 0; rho < 16; ++rho) {
      P::set(G, rho, (h == 0 && rho < 3) ? (rho == 0 ? gr.x : rho == 1 ? gr.y : gr.z) : 0.f);
      P::set(DA, rho, (h == 0 && rho == 0) ? gr.w : 0.f);
    }
    store_tile<P>(a.dz, a.nblk, ZT_TILES, ZT_RGB, wblock, lane, G);
    store_tile<P>(a.dz, a.nblk, ZT_TILES, ZT_A, wblock, lane, DA);
    {
      constexpr int N0 = [] {
        int n = 2 * CH;
        for (int j = 1; j < PF && j < GT::t.n; ++j) n += group_dma<P, 1, false>(j);
        return n;
      }();
      wait_barrier<N0>();
    }
#pragma unroll
    for (int i = 0; i < MASK_GROUPS; ++i) {
      settle(mk[i].x);
      settle(mk[i].y);
      settle(mk[i].z);
      settle(mk[i].w);
    }
    sfor<GT::t.n>([&](auto gg) { step<decltype(gg)::value>(); });
  }
};

// ------------------------------------------------------------------------------------
// The wide dX (round 6, PF32W / PBF3W): DxWave's W^T chain over 16-row units (DIR 3) on the 16x16 MFMAs, 16
// samples per wave, 8 waves per workgroup, two per SIMD.  The same register trick as FwdWave16 (a 16-row output
// tile IS half of the next stage's K-block), the forward's ReLU masks read from the old-layout lane of this
// lane's sample and half (lold), and the dZ stores in the old tile-block layout (the dW is unchanged): lane
// (s, g)'s four values of output tile m are old lane lold's registers 4 (2 (m & 1) + (g >> 1)) + e.
// ------------------------------------------------------------------------------------
template <class P>
struct DxWave16 {
  using Tile = typename P::Tile;
  using Acc = f32x4;
  static constexpr bool F32 = P::KIND == K_F32W, B16 = P::KIND == K_BF16W;
  static_assert(wide_kind<P>(), "DxWave16: PF32W, PBF3W or PBF16W");
  static constexpr int CH = P::CH;
  static constexpr int SCH = B16 ? 2 : 4;   // chunks of a stored dZ tile-block (fp32, bf16x3 hi + lo, bf16)
  static constexpr int SST = B16 || F32 ? 1 : 2;  // stores per output tile: 16-byte (fp32), hi [+ lo] 8-byte
  using GT = GroupTable<3, false, P::CH>;
  static_assert(finish_schedule_violation<P, 3, false>() == 0,
                "finish placement (NERF_FINISH_PARTS_* / NERF_FINISH_DELAY) reads a tile pair before its finish part "
                "writes it, or reads a reassigned pend (FinishSchedule)");

  const DxArgs& a;
  uint32_t lds_base;
  int lane, wave, s, g;
  int64_t m, wb32;
  uint32_t st_off, lold, gsh;
  Tile G, DA, Ha[8], Hb[8];
  uint4 mk[MASK_GROUPS];
  Acc pend;
  DmaLean dl;

  __device__ __forceinline__ DxWave16(const DxArgs& args, const uint4* smem) : a(args) {
    lds_base = (uint32_t)(uintptr_t)(lds_void*)smem;
    lane = threadIdx.x & 63;
    wave = threadIdx.x >> 6;
    s = lane & 15;
    g = lane >> 4;
    m = ((int64_t)blockIdx.x * P::WAVES + wave) * 16 + s;
    wb32 = (int64_t)blockIdx.x * (P::WAVES / 2) + (wave >> 1);
    lold = 16u * (uint32_t)(wave & 1) + (uint32_t)s + 32u * (uint32_t)(g & 1);
    st_off = 16u * lold + (F32 ? 1024u : 8u) * (uint32_t)(g >> 1);
    gsh = 2u * (uint32_t)(g >> 1);
    dl = DmaLean{a.wpack_t, (uint32_t)(lane * 16 + wave * 1024),
                 (uint32_t)__builtin_amdgcn_readfirstlane(lds_base + (uint32_t)wave * 1024u),
                 (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)wave)};
  }

  template <int gi> __device__ __forceinline__ void fetch() {
    constexpr Group Gr = GT::t.g[gi];
    fetch_group_lean<P, Gr.c0, Gr.nch, (gi % NSLOT) * SLOT_CAP * 1024>(dl);
  }
  template <int gi, int i> __device__ __forceinline__ void fetch_piece() {
    constexpr Group Gr = GT::t.g[gi];
    fetch_piece_lean<P, Gr.c0, Gr.nch, (gi % NSLOT) * SLOT_CAP * 1024, i>(dl);
  }
  static __host__ __device__ constexpr int unit_stores(int) { return SST; }
  static __host__ __device__ constexpr int group_stores(int gi) {
    int n = 0;
    for (int u = 0; u < NUNIT_BWD16; ++u)
      if (finished_in_group<3, false, P::CH, cross_finish<P, 3>()>(gi, u)) n += SST;
    return n;
  }
  template <int S> __device__ __forceinline__ Tile& slot() {
    if constexpr (S >= TS_HA && S < TS_HB) return Ha[S - TS_HA];
    else if constexpr (S >= TS_HB && S < TS_X) return Hb[S - TS_HB];
    else if constexpr (S == TS_G) return G;
    else {
      static_assert(S == TS_DA, "dX tile slot");
      return DA;
    }
  }
  static __host__ __device__ constexpr int stage_of(int u) { return bwd16_unit_stage(u); }

  // half hf of the 32-feature dZ tile tau (old layout): fp32 values v[4 hf .. 4 hf + 3], or the bf16x3 hi / lo dwords
  // 2 hf, 2 hf + 1 (8 bytes each, lo 2 KiB after hi)
  __device__ __forceinline__ void store_half(int tau, int hf, const Tile& t) {
    if constexpr (F32) {
      char* base = (char*)a.dz + (((wb32 * ZT_TILES + tau) * SCH + 2 * hf) << 10) + st_off;
      store16<0>((uint4*)base, make_uint4(__float_as_uint(t.v[4 * hf]), __float_as_uint(t.v[4 * hf + 1]),
                                          __float_as_uint(t.v[4 * hf + 2]), __float_as_uint(t.v[4 * hf + 3])));
    } else {
      char* base = (char*)a.dz + (((wb32 * ZT_TILES + tau) * SCH + hf) << 10) + st_off;
      store8(base, get_dword(t.hi, 2 * hf), get_dword(t.hi, 2 * hf + 1));
      if constexpr (!B16) store8(base + 2048, get_dword(t.lo, 2 * hf), get_dword(t.lo, 2 * hf + 1));
    }
  }

  // ---- group_body hooks
  template <int u, int t> __device__ __forceinline__ const Tile& in_tile() {
    return slot<bwd_in_slot(stage_of(u), t)>();
  }
  template <int u> __device__ __forceinline__ void prefetch() {}
  template <int u> __device__ __forceinline__ void init(Acc& acc) {
    acc[0] = acc[1] = acc[2] = acc[3] = 0.f;
  }
  // part p of NP of unit u (half m & 1 of output tile j = m >> 1 of stage st): its register pairs masked by the
  // forward's ReLU bits into the output-gradient K-block (in place); the last part stores
  template <int u, int p> __device__ __forceinline__ void finish_part(const Acc& acc) {
    constexpr int st = stage_of(u), mu = u - bwd16_unit_first(st), j = mu >> 1, hf = mu & 1;
    constexpr int mg = bwd_mask_group(st);
    constexpr int NP = finish_parts<P>();
    constexpr int K0 = 2 * p / NP, K1 = 2 * (p + 1) / NP;
    uint32_t w = 0xFFFFFFFFu;
    if constexpr (mg >= 0) {
      // value e (pair k = e >> 1, element e & 1) of this lane: old register rho = 4 (2 hf + (g >> 1)) + e of old
      // tile j, mask bit 8 (j & 1) + (rho >> 1) + 16 (rho & 1) = [k + 16 (e & 1)] << (8 (j & 1) + 4 hf + gsh)
      const uint32_t d = (j >> 1) == 0 ? mk[mg].x : (j >> 1) == 1 ? mk[mg].y : (j >> 1) == 2 ? mk[mg].z : mk[mg].w;
      w = d >> ((uint32_t)(8 * (j & 1) + 4 * hf) + gsh);
    }
    Tile& out = slot<bwd_out_slot(st, j)>();
    sfor<K1 - K0>([&](auto kk) {
      constexpr int k = K0 + decltype(kk)::value;
      const float y0 = ((w >> k) & 1u) ? acc[2 * k] : 0.f;
      const float y1 = ((w >> (16 + k)) & 1u) ? acc[2 * k + 1] : 0.f;
      if constexpr (F32) {
        out.v[4 * hf + 2 * k] = y0;
        out.v[4 * hf + 2 * k + 1] = y1;
      } else if constexpr (B16) {
        set_dword8(out.hi, 2 * hf + k, pack_bf16(y0, y1));
      } else {
        const uint32_t hw = pack_bf16(y0, y1);
        const uint32_t lw = pack_bf16(y0 - __uint_as_float(hw << 16), y1 - __uint_as_float(hw & 0xffff0000u));
        set_dword8(out.hi, 2 * hf + k, hw);
        set_dword8(out.lo, 2 * hf + k, lw);
      }
    });
    if constexpr (p == NP - 1) store_half(bwd_dz_tile(st, j), hf, out);
  }

  template <int gi> __device__ __forceinline__ void step() {
    constexpr int NG = GT::t.n;
    if constexpr (gi + PF < NG && dma_spread<P>() == 0) fetch<gi + PF>();
    const uint32_t sl = lds_base + (uint32_t)((gi % NSLOT) * SLOT_CAP * 1024);
    group_body<P, 3, false, gi>(*this, lds_ptr(sl + (uint32_t)(lane * 16)));
    constexpr int N = dma_spread<P>() > 0
        ? handoff_vmcnt_spread<P, 3, false>(gi, [](int u) constexpr { return unit_stores(u); })
        : handoff_vmcnt<P, 3, false>(gi, [](int i) constexpr { return group_stores(i); }, 4 * SST);
    if constexpr (gi + 1 < NG) wait_barrier<N>();
  }

  // the seed tiles: K-block 0 of d rgb (features 0..2) and of d alpha (feature 0), element e of lane group g =
  // feature k16_feat(g, e): lane group 0's elements 0..2 / 0
  __device__ __forceinline__ void seed(Tile& t, float v0, float v1, float v2) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    if (g == 0) v[0] = v0, v[1] = v1, v[2] = v2;
    if constexpr (F32) {
#pragma unroll
      for (int e = 0; e < 8; ++e) t.v[e] = v[e];
    } else {
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hw[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
        lw[k] = pack_bf16(v[2 * k] - __uint_as_float(hw[k] << 16), v[2 * k + 1] - __uint_as_float(hw[k] & 0xffff0000u));
      }
      t.hi = __builtin_bit_cast(bf16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
      if constexpr (!B16) t.lo = __builtin_bit_cast(bf16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
    }
  }

  __device__ __forceinline__ void run() {
    const float4 gr = m < a.M ? *(const float4*)(a.d_raw + m * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < MASK_GROUPS; ++i) mk[i] = *mask_slot((void*)a.masks, wb32, i, (int)lold);
    sfor<(PF < GT::t.n ? PF : GT::t.n)>([&](auto gg) { fetch<decltype(gg)::value>(); });
    seed(G, gr.x, gr.y, gr.z);
    seed(DA, gr.w, 0.f, 0.f);
    store_half(ZT_RGB, 0, G);
    store_half(ZT_RGB, 1, G);
    store_half(ZT_A, 0, DA);
    store_half(ZT_A, 1, DA);
    {
      constexpr int N0 = [] {
        int n = 4 * SST;
        for (int j = 1; j < PF && j < GT::t.n; ++j) n += group_dma<P, 3, false>(j);
        return n;
      }();
      wait_barrier<N0>();
    }
#pragma unroll
    for (int i = 0; i < MASK_GROUPS; ++i) {
      settle(mk[i].x);
      settle(mk[i].y);
      settle(mk[i].z);
      settle(mk[i].w);
    }
    sfor<GT::t.n>([&](auto gg) { step<decltype(gg)::value>(); });
  }
};

template <class P>
using DxWaveOf = std::conditional_t<wide_kind<P>(), DxWave16<P>, DxWave<P>>;

template <class P>
__global__ void __launch_bounds__(P::WAVES * 64) dx_kernel(DxArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem_u4[];
  DxWaveOf<P> w(a, smem_u4);
  w.run();
}

// ------------------------------------------------------------------------------------
// dW / db: C[n][k] += sum_m dz[n][m] act[k][m] (K = samples), one pass over the stores.
//
// Ten jobs, each reading every tile it needs once per 32-sample block (159 tile-blocks per
// block for the whole net):
//   J0..J7  pts_linears.l: 8 dZ_l tiles x (2 | 8 | 10) act tiles; wave w owns n-tile w
//   J8      feature_linear (8 dF x 8 h7) + alpha_linear (dA x h7): wave w also owns the
//           alpha row against h7 tile w
//   J9      views_linears (4 dZv x [8 feature, PE(dir)]) on waves 0..3 + rgb_linear
//           (d rgb x hv tile w-4) on waves 4..7
// Work items = (job, contiguous block range) sized to equal bytes, as many as there are
// CUs (nerf_mlp_dw_items), so the single wave of workgroups ends together.  Per block, a
// job's tile-blocks (fragment-native, mlp_tables.h) stream into an LDS ring with LDS-DMA
// and are read back transposed (ds_read_b64_tr_b16): row i of a fragment <-> feature
// acc_row(i & 15, i >> 4).  Each item adds its partial sums with fp32 atomics.
// ------------------------------------------------------------------------------------
constexpr int DW_WAVES = 8;
constexpr int DW_SLOTS = 18;  // most tile-blocks one job reads per block
constexpr int NDWJOB = 10;
enum DwKind { DW_REG = 0, DW_FA = 1, DW_VR = 2 };

struct DwJobDesc {
  int kind, kt;     // kind; k-tiles per wave (REG / FA trunk / VR view waves)
  int nd, na;       // dz tiles, act tiles (LDS slots [0, nd) then [nd, nd + na))
  int dz[9];        // dz tile ids
  int act[13];      // act tile ids
};
__host__ __device__ constexpr DwJobDesc dw_job_desc(int j) {
  DwJobDesc d{};
  if (j < 8) {
    d.kind = DW_REG;
    d.kt = gemm_k_tiles(j);
    d.nd = 8;
    d.na = d.kt;
    for (int n = 0; n < 8; ++n) d.dz[n] = ZT_H + 8 * j + n;
    for (int t = 0; t < d.kt; ++t) d.act[t] = gemm_act_tile(j, t);
  } else if (j == 8) {
    d.kind = DW_FA;
    d.kt = 8;
    d.nd = 9;
    d.na = 8;
    for (int n = 0; n < 8; ++n) d.dz[n] = ZT_F + n;
    d.dz[8] = ZT_A;
    for (int t = 0; t < 8; ++t) d.act[t] = AT_H + 56 + t;
  } else {
    d.kind = DW_VR;
    d.kt = 9;
    d.nd = 5;
    d.na = 13;
    for (int n = 0; n < 4; ++n) d.dz[n] = ZT_V + n;
    d.dz[4] = ZT_RGB;
    for (int t = 0; t < 8; ++t) d.act[t] = AT_F + t;
    d.act[8] = AT_D;
    for (int t = 0; t < 4; ++t) d.act[9 + t] = AT_V + t;
  }
  return d;
}
__host__ __device__ constexpr int dw_job_tiles(int j) { return dw_job_desc(j).nd + dw_job_desc(j).na; }

// LDS ring depth: 4 x 36 KiB (bf16), 2 x 72 KiB (fp32)
#ifndef NERF_DW_NBUF_BF16
#define NERF_DW_NBUF_BF16 4
#endif
template <class P> __host__ __device__ constexpr int dw_nbuf() { return P::KIND == K_BF16 ? NERF_DW_NBUF_BF16 : 2; }
__host__ __device__ constexpr int perm_row(int i) { return acc_row(i & 15, i >> 4); }

// work items: segment s = items [item_off[s], item_off[s + 1]) of job job_of[s]
// (item_off[NDWJOB] = total); segments are ordered longest item first
struct DwArgs {
  const void* dz;
  const void* act;
  int64_t nblk;       // 32-sample blocks in the stores
  float* grad;        // flat [NET_PARAMS], accumulated
  int item_off[NDWJOB + 1];
  int job_of[NDWJOB];
  float* partial;     // per-item partial sums (deterministic mode, dw_reduce_kernel) or null (atomics)
};

// Deterministic mode: every work item writes its accumulators, fragment-native, to its own
// slice of `partial` -- per wave DW_PSLOTS tiles (acc[0..9] -> 0..9, acc2 -> 10) of 64 lanes x
// 16 floats, then 128 floats of row sums (dbias lanes 0..63, dbias2 lanes 0..63) -- and
// dw_reduce_kernel adds the items of each job in item order: the same sum on every run.
constexpr int DW_PSLOTS = 11;
constexpr int DW_PWAVE = DW_PSLOTS * 1024 + 128;   // floats per wave
constexpr int DW_PITEM = DW_WAVES * DW_PWAVE;      // floats per item

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 63] (n is a multiple of G here)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
#define NERF_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    NERF_VMW(0) NERF_VMW(1) NERF_VMW(2) NERF_VMW(3) NERF_VMW(4) NERF_VMW(5) NERF_VMW(6) NERF_VMW(7)
    NERF_VMW(8) NERF_VMW(9) NERF_VMW(10) NERF_VMW(11) NERF_VMW(12) NERF_VMW(13) NERF_VMW(14) NERF_VMW(15)
    NERF_VMW(16) NERF_VMW(17) NERF_VMW(18)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
#undef NERF_VMW
}

typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((address_space(3))) short4_t lds_short4;

// bf16 LDS swizzle of the dW ring.  A stored chunk is 64 lane-linear 16-B pieces; the
// transposed fragment read below touches pieces p = 16 a + b with b in {q, q + 4} (+ 8 for
// lanes 32..63), a in {s, s + 2}, of both chunks of a tile at once -- 16 of the 64 banks
// as stored.  Piece p of chunk c is placed at slot 16 a + (b + 4 (a >> 1) + 8 c) mod 16
// instead (the DMA's per-lane source address does the permutation for free), which makes
// every ds_read_b64_tr_b16 conflict-free.
__host__ __device__ constexpr int dw_swz(int c, int p) {
  return 16 * (p >> 4) + (((p & 15) + 4 * ((p >> 4) >> 1) + 8 * c) & 15);
}
__host__ __device__ constexpr int dw_unswz(int c, int slot) {
  return 16 * (slot >> 4) + (((slot & 15) - 4 * ((slot >> 4) >> 1) - 8 * c) & 15);
}

// bf16: the 8-sample K fragment (samples 16 s + 8 h + [0, 8)) of row (lane & 31)
__device__ __forceinline__ bf16x8 dw_frag_bf16(const char* tile, int s, int lane) {
  const int l16 = lane & 15, G = lane >> 4;
  const int hp = G & 1, h = G >> 1, q = l16 >> 2, pp = l16 & 3;
  const int c = pp >> 1, p = 16 * s + 8 * h + q + 32 * hp;
  const char* base = tile + c * 1024 + (pp & 1) * 8;
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(base + dw_swz(c, p) * 16));
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(base + dw_swz(c, p + 4) * 16));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
// fp32 LDS swizzle of the dW ring.  The K = 2 fragment read below has the 32 lanes of one
// ds_read_b32 bank group touch pieces p in {2 s + h, 2 s + h + 32} of all 4 chunks (dword
// rho & 3 of each): as stored, those 8 pieces sit at the same (slot mod 8), i.e. on 4 of the
// 32 banks -- an 8-way conflict.  Piece p of chunk c is placed at slot
// (p & ~7) | ((p + 2 c + (p >> 5)) & 7) instead, which puts the 8 pieces on 8 distinct
// (slot mod 8) and every read conflict-free.
__host__ __device__ constexpr int dw_swz_f32(int c, int p) { return (p & ~7) | ((p + 2 * c + (p >> 5)) & 7); }
__host__ __device__ constexpr int dw_unswz_f32(int c, int q) { return (q & ~7) | ((q - 2 * c - (q >> 5)) & 7); }

// fp32: the K = 2 fragment (sample 2 s + h) of row (lane & 31).  With s = 4 a + b, the slot
// dw_swz_f32(c, 2 s + h + 32 hp) = 8 a + 32 hp + ((2 b + h + 2 c + hp) & 7): the per-lane part
// depends on s & 3 only.  A tile region's four per-lane bases (F32Base) are laundered through
// empty asm, so every read is one ds_read_b32 at base + immediate (tile * 4 KiB + 128 a).
#ifndef NERF_DW_SWZ_F32
#define NERF_DW_SWZ_F32 1
#endif
__device__ __forceinline__ uint32_t dw_f32_lane_off(int lane, int b) {
  const int rho = lane & 15, hp = (lane >> 4) & 1, h = lane >> 5, c = rho >> 2;
  const int sw = NERF_DW_SWZ_F32 ? 2 * c + hp : 0;
  return (uint32_t)(c * 1024 + 512 * hp + 16 * ((2 * b + h + sw) & 7) + 4 * (rho & 3));
}
struct F32Base { uint32_t b[4]; };
__device__ __forceinline__ F32Base f32_base(uint32_t region, const uint32_t (&lane_off)[4]) {
  F32Base r;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    r.b[b] = region + lane_off[b];
    settle(r.b[b]);
  }
  return r;
}
typedef __attribute__((address_space(3))) const float lds_cf;
template <int IMM>
__device__ __forceinline__ float f32_frag(const F32Base& B, int s) {
  static_assert(IMM >= 0 && IMM + 128 * 3 < 65536, "ds_read offset is 16 bits");
  return *(lds_cf*)(uintptr_t)(B.b[s & 3] + (uint32_t)(IMM + 128 * (s >> 2)));
}
#ifndef NERF_DW_F32_PIPE
#define NERF_DW_F32_PIPE 1
#endif
// step after which the pipelined fp32 K loop issues the next block's DMA (-1: before the loop),
// waves 4..7 NERF_DW_FETCH_SPLIT steps later (after step 1 / step 5: 5.05 -> 4.95 ms at 524k samples)
#ifndef NERF_DW_FETCH_STEP
#define NERF_DW_FETCH_STEP 1
#endif
#ifndef NERF_DW_FETCH_SPLIT
#define NERF_DW_FETCH_SPLIT 4
#endif
__device__ __forceinline__ float dw_frag_f32(const char* tile, int s, int lane) {
  return *(const float*)(tile + dw_f32_lane_off(lane, s & 3) + 128 * (s >> 2));
}

// one K step (16 samples bf16 / 2 samples fp32) of C += A B^T for A = LDS tile `at`
template <class P>
__device__ __forceinline__ f32x16 dw_mma(const char* at, const char* bt, int s, int lane, f32x16 acc) {
  if constexpr (P::KIND == K_BF16) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(dw_frag_bf16(at, s, lane), dw_frag_bf16(bt, s, lane), acc, 0, 0, 0);
  } else if constexpr (P::KIND == K_BF16X3) {  // tile-block = hi (2 KiB) then lo (2 KiB)
    const bf16x8 ah = dw_frag_bf16(at, s, lane), al = dw_frag_bf16(at + 2048, s, lane);
    const bf16x8 bh = dw_frag_bf16(bt, s, lane), bl = dw_frag_bf16(bt + 2048, s, lane);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  } else {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(dw_frag_f32(at, s, lane), dw_frag_f32(bt, s, lane), acc, 0, 0, 0);
  }
}
template <class P>
__device__ __forceinline__ float dw_rowsum(const char* at, int s, int lane) {
  if constexpr (P::KIND != K_F32) {
    const bf16x8 v = dw_frag_bf16(at, s, lane);
    float r = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) r += (float)v[e];
    if constexpr (P::KIND == K_BF16X3) {
      const bf16x8 l = dw_frag_bf16(at + 2048, s, lane);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (float)l[e];
      r += q;
    }
    return r;
  } else {
    return dw_frag_f32(at, s, lane);
  }
}

// add a 32 x 32 accumulator tile into weight WP at rows 32 ntile + perm, columns col0 +
// perm (valid rows < nvalid, valid columns < cvalid of the tile).  The layout functions
// are loops: every use sits in a constant expression.
template <int WP>
__device__ __forceinline__ void dw_flush(float* grad, int ntile, int nvalid, int col0, int cvalid, const f32x16& acc,
                                         int lane) {
  constexpr int64_t OFF = param_offset(WP);
  constexpr int K = weight_K(WP);
  float* gw = grad + OFF;
  const int h = lane >> 5, colf = perm_row(lane & 31);
  if (colf >= cvalid) return;
#pragma unroll
  for (int rho = 0; rho < 16; ++rho) {
    const int n = 32 * ntile + perm_row(acc_row(rho, h));
    if (n < nvalid) atomicAdd(gw + (int64_t)n * K + col0 + colf, acc[rho]);
  }
}
template <int WPB>
__device__ __forceinline__ void dw_flush_bias(float* grad, int ntile, int nvalid, float dbias, int lane) {
  constexpr int64_t OFF = param_offset(WPB);
  dbias += __shfl_xor(dbias, 32, 64);
  const int n = 32 * ntile + perm_row(lane & 31);
  if (lane < 32 && n < nvalid) atomicAdd(grad + OFF + n, dbias);
}

// LDS slot of job tile q (q < nd: dz tile q, else act tile q - nd): the act tiles come first,
// so a K step's act-tile reads are one per-lane base + immediates below 64 KiB
__host__ __device__ constexpr int dw_slot(const DwJobDesc& d, int q) { return q < d.nd ? d.na + q : q - d.nd; }

// dW's tile stream is read exactly once (each tile-block by one work item), so it is loaded nt
// (bf16 dW 0.957 -> 0.926 ms, bf16x3 2.05 -> 2.02 at 524,288 samples; fp32 unchanged)
#ifndef NERF_DW_DMA_NT
#define NERF_DW_DMA_NT 1
#endif
#if NERF_DW_DMA_NT
#define NERF_DW_DMA_AUX " nt"
#else
#define NERF_DW_DMA_AUX ""
#endif
// global_load_lds_dwordx4 with a uniform 64-bit base (SGPR pair) + per-lane 32-bit offset
// (the SADDR form: one VGPR per fetch stream instead of a 64-bit address pair)
__device__ __forceinline__ void glds16_saddr(const void* sbase, uint32_t voff, uint32_t lds_wave_base) {
  uint32_t saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" NERF_DW_DMA_AUX "\n\ts_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(voff), "s"(sbase), "s"(__builtin_amdgcn_readfirstlane(lds_wave_base)) : "memory");
}

// a wave-uniform pointer made visibly uniform (SGPR pair) to the compiler
__device__ __forceinline__ const char* uniform_ptr(const char* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const char*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

template <class P, int J>
__device__ __forceinline__ void dw_job(const DwArgs& a, int64_t b_begin, int64_t b_end, char* lds) {
  constexpr DwJobDesc JD = dw_job_desc(J);
  constexpr int TB = P::CH * 1024;            // tile-block bytes
  constexpr int BUF = DW_SLOTS * TB;          // one stage of the ring
  constexpr int NT = JD.nd + JD.na;
  constexpr int NCHUNK = NT * P::CH;
  constexpr int G = (NCHUNK + DW_WAVES - 1) / DW_WAVES;  // DMA per wave per block (uniform)
  constexpr int NBUF = dw_nbuf<P>(), D = NBUF - 1;
  constexpr int KS = P::KIND == K_F32 ? 16 : 2;  // K steps per 32-sample block
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;  // (kept divergent to the compiler: uniform branching spills)

  // DMA streams, resolved once (a table lookup inside the loop would be a compiler-visible
  // load, whose wait drains the ring): uniform tile base (block 0) + per-lane piece offset
  const char* sb[G];
  uint32_t voff[G];
  uint32_t dst[G];
  int64_t bstride[G];
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const int k = cmin(wave + DW_WAVES * i, NCHUNK - 1);
    const int q = k / P::CH, c = k % P::CH;
    const bool is_dz = q < JD.nd;
    int tau = 0;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (t == q) tau = t < JD.nd ? JD.dz[t] : JD.act[t - JD.nd];
    const int ntiles = is_dz ? ZT_TILES : AT_TILES;
    // swizzled rings (bf16x3: chunks 2, 3 are the lo tile, swizzled as chunks 0, 1)
    const int piece = P::KIND != K_F32 ? dw_unswz(c & 1, lane) : NERF_DW_SWZ_F32 ? dw_unswz_f32(c, lane) : lane;
    sb[i] = uniform_ptr((const char*)(is_dz ? a.dz : a.act) + tile_kib(a.nblk, ntiles, tau, 0, c, P::CH) * 1024);
    voff[i] = (uint32_t)(piece * 16);
    bstride[i] = block_stride_kib(ntiles, P::CH) * 1024;
    int slot = 0;
#pragma unroll
    for (int t = 0; t < NT; ++t)
      if (t == q) slot = dw_slot(JD, t);
    dst[i] = (uint32_t)(slot * TB + c * 1024);
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void*)lds;
  auto fetch = [&](int64_t b, int buf) {
#pragma unroll
    for (int i = 0; i < G; ++i)
      glds16_saddr(uniform_ptr(sb[i] + b * bstride[i]), voff[i], lds_base + (uint32_t)(buf * BUF) + dst[i]);
  };

  // wave roles
  //   REG: dz tile w x act tiles 0 .. kt;  FA: + alpha (dz tile 8) x act tile w
  //   VR: waves 0..3 dz tile w x act tiles 0 .. 9; waves 4..7 d rgb (dz tile 4) x act tile 9 + (w - 4)
  const bool vr_rgb = JD.kind == DW_VR && wave >= 4;
  const int n_q = vr_rgb ? 4 : wave;         // dz tile of this wave
  const int n_lds = JD.na + n_q;             // its LDS slot
  f32x16 acc[10], acc2;
#pragma unroll
  for (int t = 0; t < 10; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc2[i] = 0.f;
  float dbias = 0.f, dbias2 = 0.f;
  uint32_t lane_off[4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) lane_off[bb] = dw_f32_lane_off(lane, bb);

  for (int d = 0; d < D; ++d)
    if (b_begin + d < b_end) fetch(b_begin + d, d);
  int buf = 0;
  for (int64_t b = b_begin; b < b_end; ++b) {
    const int younger = (int)min((int64_t)(D - 1), b_end - 1 - b);
    wait_vmcnt_rt(G * younger);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // fp32 (pipelined): the next block's DMA is issued inside the K loop (NERF_DW_FETCH_STEP), the two
    // waves of a SIMD (w, w + 4) at different steps, so its ~70 issue slots overlap the partner's MFMAs
    constexpr bool FETCH_IN_LOOP = P::KIND == K_F32 && NERF_DW_F32_PIPE && NERF_DW_FETCH_STEP >= 0;
    const int fbuf = buf == 0 ? NBUF - 1 : buf - 1;
    if (!FETCH_IN_LOOP && b + D < b_end) fetch(b + D, fbuf);
    const char* tiles = lds + buf * BUF;
    if constexpr (P::KIND == K_F32 && NERF_DW_F32_PIPE) {
      // 16 K steps, fully unrolled, software-pipelined one step deep: step s + 1's fragments
      // (the dz fragment, the k-tiles' act fragments, the alpha pair) are read before step
      // s's MFMAs issue, fenced by sched_barrier so hipcc keeps that order (on its own it read
      // two fragments, waited lgkmcnt(0), issued two MFMAs: every LDS latency exposed).
      // Every read is one of four per-lane bases (s & 3) + an immediate (< 64 KiB).
      constexpr int KT = JD.kind == DW_VR ? 9 : JD.kt;
      constexpr int NF = 1 + KT + (JD.kind == DW_FA ? 2 : 0);
      const uint32_t region = lds_base + (uint32_t)(buf * BUF);
      const F32Base Bn = f32_base(region + (uint32_t)(n_lds * TB), lane_off);
      // act tiles: all of them from slot 0 (immediates t * 4 KiB), or the rgb wave's one
      const F32Base Ba = f32_base(region + (uint32_t)(vr_rgb ? (9 + wave - 4) * TB : 0), lane_off);
      F32Base Bal{}, Bw{};
      if constexpr (JD.kind == DW_FA) {
        Bal = f32_base(region + (uint32_t)((JD.na + 8) * TB), lane_off);
        Bw = f32_base(region + (uint32_t)(wave * TB), lane_off);
      }
      float fr[2][NF];
      auto rd = [&](auto ss, float (&f)[NF]) {
        constexpr int s = decltype(ss)::value;
        constexpr int SOFF = 128 * (s >> 2);
        f[0] = f32_frag<SOFF>(Bn, s & 3);
        if (!vr_rgb) {
          sfor<KT>([&](auto tt) {
            constexpr int t = decltype(tt)::value;
            f[1 + t] = f32_frag<t * TB + SOFF>(Ba, s & 3);
          });
        } else {
          f[1] = f32_frag<SOFF>(Ba, s & 3);
        }
        if constexpr (JD.kind == DW_FA) {
          f[KT + 1] = f32_frag<SOFF>(Bal, s & 3);
          f[KT + 2] = f32_frag<SOFF>(Bw, s & 3);
        }
      };
      auto mm = [&](const float (&f)[NF]) {
        dbias += f[0];
        if (!vr_rgb) {
          sfor<KT>([&](auto tt) {
            constexpr int t = decltype(tt)::value;
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(f[0], f[1 + t], acc[t], 0, 0, 0);
          });
        } else {
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(f[0], f[1], acc[0], 0, 0, 0);
        }
        if constexpr (JD.kind == DW_FA) {
          if (wave == 0) dbias2 += f[KT + 1];
          acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(f[KT + 1], f[KT + 2], acc2, 0, 0, 0);
        }
      };
      rd(std::integral_constant<int, 0>{}, fr[0]);
      const bool fhi = wave >= 4;
      sfor<16>([&](auto ss) {
        constexpr int s = decltype(ss)::value;
        if constexpr (s + 1 < 16) rd(std::integral_constant<int, s + 1>{}, fr[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mm(fr[s & 1]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (FETCH_IN_LOOP && s == NERF_DW_FETCH_STEP) {
          if (!fhi && b + D < b_end) fetch(b + D, fbuf);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (FETCH_IN_LOOP && s == NERF_DW_FETCH_STEP + NERF_DW_FETCH_SPLIT) {
          if (fhi && b + D < b_end) fetch(b + D, fbuf);
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    } else if constexpr (P::KIND == K_F32) {
      // 16 K steps as 4 rounds of 4 (s = 4 a + b): the rounds are a real loop (the bases step
      // by 128 B), so the scheduler's window -- and the fragments it keeps in flight -- is
      // one round, not the whole block
      const uint32_t region = lds_base + (uint32_t)(buf * BUF);
      uint32_t rn = region + (uint32_t)(n_lds * TB);
      // act tiles: all of them from slot 0 (immediates t * 4 KiB), or the rgb wave's one
      uint32_t ra = region + (uint32_t)(vr_rgb ? (9 + wave - 4) * TB : 0);
      uint32_t ral = region + (uint32_t)((JD.na + 8) * TB), rw = region + (uint32_t)(wave * TB);
#pragma nounroll
      for (int ar = 0; ar < 4; ++ar) {
        const F32Base Bn = f32_base(rn, lane_off), Ba = f32_base(ra, lane_off);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float an = f32_frag<0>(Bn, s);
          dbias += an;
          if (!vr_rgb) {
            sfor<JD.kt>([&](auto tt) {
              constexpr int t = decltype(tt)::value;
              acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(an, f32_frag<t * TB>(Ba, s), acc[t], 0, 0, 0);
            });
          } else {
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(an, f32_frag<0>(Ba, s), acc[0], 0, 0, 0);
          }
        }
        if constexpr (JD.kind == DW_FA) {
          const F32Base Bal = f32_base(ral, lane_off), Bw = f32_base(rw, lane_off);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float al = f32_frag<0>(Bal, s);
            if (wave == 0) dbias2 += al;
            acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(al, f32_frag<0>(Bw, s), acc2, 0, 0, 0);
          }
        }
        rn += 128;
        ra += 128;
        ral += 128;
        rw += 128;
      }
    } else {
      const char* nt = tiles + n_lds * TB;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        if (!vr_rgb) {
          dbias += dw_rowsum<P>(nt, s, lane);
#pragma unroll
          for (int t = 0; t < JD.kt; ++t) acc[t] = dw_mma<P>(nt, tiles + t * TB, s, lane, acc[t]);
        } else {
          dbias += dw_rowsum<P>(nt, s, lane);
          acc[0] = dw_mma<P>(nt, tiles + (9 + (wave - 4)) * TB, s, lane, acc[0]);
        }
        if constexpr (JD.kind == DW_FA) {
          const char* at = tiles + (JD.na + 8) * TB;
          if (wave == 0) dbias2 += dw_rowsum<P>(at, s, lane);
          acc2 = dw_mma<P>(at, tiles + wave * TB, s, lane, acc2);
        }
      }
    }
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }

  if (a.partial) {  // deterministic: the item's sums to its own slice (dw_reduce_kernel adds them)
    float* pw = a.partial + ((int64_t)blockIdx.x * DW_WAVES + wave) * DW_PWAVE;
    auto put = [&](int slot, const f32x16& v) {
      float* d = pw + slot * 1024 + lane * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) *(float4*)(d + q * 256) = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    };
    constexpr int NACC = JD.kind == DW_VR ? 9 : JD.kt;
    if (!vr_rgb) {
      sfor<NACC>([&](auto tt) { put(decltype(tt)::value, acc[decltype(tt)::value]); });
    } else {
      put(0, acc[0]);
    }
    if constexpr (JD.kind == DW_FA) put(10, acc2);
    pw[DW_PSLOTS * 1024 + lane] = dbias;
    pw[DW_PSLOTS * 1024 + 64 + lane] = dbias2;
    return;
  }
  // flush (state_dict layout: weight [N][K] row-major)
  if constexpr (JD.kind == DW_REG) {
    constexpr int WP = gemm_weight(J);
    sfor<JD.kt>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      constexpr int C0 = gemm_col0(J, t), CV = gemm_col_valid(J, t);
      dw_flush<WP>(a.grad, wave, 256, C0, CV, acc[t], lane);
    });
    dw_flush_bias<WP + 1>(a.grad, wave, 256, dbias, lane);
  } else if constexpr (JD.kind == DW_FA) {
#pragma unroll
    for (int t = 0; t < 8; ++t) dw_flush<P_FW>(a.grad, wave, 256, 32 * t, 32, acc[t], lane);
    dw_flush_bias<P_FB>(a.grad, wave, 256, dbias, lane);
    dw_flush<P_AW>(a.grad, 0, 1, 32 * wave, 32, acc2, lane);
    if (wave == 0) dw_flush_bias<P_AB>(a.grad, 0, 1, dbias2, lane);
  } else {
    if (!vr_rgb) {
#pragma unroll
      for (int t = 0; t < 9; ++t) dw_flush<P_VW>(a.grad, wave, 128, 32 * t, t < 8 ? 32 : 27, acc[t], lane);
      dw_flush_bias<P_VB>(a.grad, wave, 128, dbias, lane);
    } else {
      dw_flush<P_RW>(a.grad, 0, 3, 32 * (wave - 4), 32, acc[0], lane);
      if (wave == 4) dw_flush_bias<P_RB>(a.grad, 0, 3, dbias, lane);
    }
  }
}

template <class P>
__global__ void __launch_bounds__(DW_WAVES * 64) dw_kernel(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem_u4[];
  char* lds = (char*)smem_u4;
  const int item = blockIdx.x;
  int seg = 0;
#pragma unroll
  for (int k = 1; k < NDWJOB; ++k) seg += a.item_off[k] <= item ? 1 : 0;
  const int n_items = a.item_off[seg + 1] - a.item_off[seg], i = item - a.item_off[seg];
  const int j = a.job_of[seg];
  const int64_t b_begin = a.nblk * i / n_items, b_end = a.nblk * (i + 1) / n_items;
  switch (j) {
    case 0: dw_job<P, 0>(a, b_begin, b_end, lds); break;
    case 1: dw_job<P, 1>(a, b_begin, b_end, lds); break;
    case 2: dw_job<P, 2>(a, b_begin, b_end, lds); break;
    case 3: dw_job<P, 3>(a, b_begin, b_end, lds); break;
    case 4: dw_job<P, 4>(a, b_begin, b_end, lds); break;
    case 5: dw_job<P, 5>(a, b_begin, b_end, lds); break;
    case 6: dw_job<P, 6>(a, b_begin, b_end, lds); break;
    case 7: dw_job<P, 7>(a, b_begin, b_end, lds); break;
    case 8: dw_job<P, 8>(a, b_begin, b_end, lds); break;
    default: dw_job<P, 9>(a, b_begin, b_end, lds); break;
  }
}

// flat-gradient index of element (wave w, slot t, lane, register rho) of job J's partial
// accumulators, or -1 (padding / unused): the inverse of the dw_flush / dw_flush_bias maps.
// Slot DW_PSLOTS holds the row sums: q = element (0..127) -- q < 32: dbias of lanes q and
// q + 32 (returned for q only; the caller adds both), 64 <= q < 96: dbias2 likewise.
template <int J>
__device__ __forceinline__ int64_t dw_param_index(int w, int t, int lane, int rho) {
  constexpr DwJobDesc JD = dw_job_desc(J);
  const int h = lane >> 5, colf = perm_row(lane & 31), nrow = perm_row(acc_row(rho, h));
  if constexpr (JD.kind == DW_REG) {
    constexpr int WP = gemm_weight(J);
    if (t >= JD.kt) return -1;
    const int c0 = gemm_col0(J, t), cv = gemm_col_valid(J, t);
    if (colf >= cv) return -1;
    return param_offset(WP) + (int64_t)(32 * w + nrow) * weight_K(WP) + c0 + colf;
  } else if constexpr (JD.kind == DW_FA) {
    if (t < 8) return param_offset(P_FW) + (int64_t)(32 * w + nrow) * 256 + 32 * t + colf;
    if (t == 10 && nrow < 1) return param_offset(P_AW) + 32 * w + colf;
    return -1;
  } else {
    if (w < 4) {
      if (t >= 9 || colf >= (t < 8 ? 32 : 27)) return -1;
      return param_offset(P_VW) + (int64_t)(32 * w + nrow) * 283 + 32 * t + colf;
    }
    if (t == 0 && nrow < 3) return param_offset(P_RW) + (int64_t)nrow * 128 + 32 * (w - 4) + colf;
    return -1;
  }
}
template <int J>
__device__ __forceinline__ int64_t dw_bias_index(int w, int q) {
  constexpr DwJobDesc JD = dw_job_desc(J);
  const int n = perm_row(q & 31);
  if (q < 32) {
    if constexpr (JD.kind == DW_REG) return param_offset(gemm_weight(J) + 1) + 32 * w + n;
    else if constexpr (JD.kind == DW_FA) return param_offset(P_FB) + 32 * w + n;
    else {
      if (w < 4) return param_offset(P_VB) + 32 * w + n;
      return (w == 4 && n < 3) ? param_offset(P_RB) + n : -1;
    }
  }
  if (q >= 64 && q < 96 && JD.kind == DW_FA && w == 0 && n < 1) return param_offset(P_AB);
  return -1;
}

struct DwReduceArgs {
  const float* partial;
  float* grad;
  int item_off[NDWJOB + 1];
  int job_of[NDWJOB];
};

// one thread per (segment, wave, partial element); sums the segment's items in order
template <int J>
__device__ __forceinline__ void dw_reduce_job(const DwReduceArgs& a, int i0, int n, int w, int e) {
  int64_t idx;
  bool bias = e >= DW_PSLOTS * 1024;
  if (!bias) {
    const int t = e >> 10, r = e & 1023, q = r >> 8, lane = (r >> 2) & 63, rho = 4 * q + (r & 3);
    idx = dw_param_index<J>(w, t, lane, rho);
  } else {
    idx = dw_bias_index<J>(w, e - DW_PSLOTS * 1024);
  }
  if (idx < 0) return;
  const float* p = a.partial + ((int64_t)i0 * DW_WAVES + w) * DW_PWAVE + e;
  // row sums: lanes q and q + 32 of one item
  auto item = [&](int i) { const float* pi = p + (int64_t)i * DW_PITEM; return bias ? pi[0] + pi[32] : pi[0]; };
  // the items in order, 8 loads in flight (a one-load-per-iteration loop made the reduce a chain of n
  // dependent round trips: 21 us per launch at ~25 items per job)
  float sum = 0.f;
  int i = 0;
  for (; i + 8 <= n; i += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = item(i + k);
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += v[k];
  }
  for (; i < n; ++i) sum += item(i);
  a.grad[idx] += sum;
}

#if !defined(NERF_MLP_PREC)  // non-template: defined in the C-ABI translation unit only
__global__ void dw_reduce_kernel(DwReduceArgs a) {
  const int seg = blockIdx.y;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (int64_t)DW_WAVES * DW_PWAVE) return;
  const int w = (int)(g / DW_PWAVE), e = (int)(g % DW_PWAVE);
  const int i0 = a.item_off[seg], n = a.item_off[seg + 1] - i0;
  switch (a.job_of[seg]) {
    case 0: dw_reduce_job<0>(a, i0, n, w, e); break;
    case 1: dw_reduce_job<1>(a, i0, n, w, e); break;
    case 2: dw_reduce_job<2>(a, i0, n, w, e); break;
    case 3: dw_reduce_job<3>(a, i0, n, w, e); break;
    case 4: dw_reduce_job<4>(a, i0, n, w, e); break;
    case 5: dw_reduce_job<5>(a, i0, n, w, e); break;
    case 6: dw_reduce_job<6>(a, i0, n, w, e); break;
    case 7: dw_reduce_job<7>(a, i0, n, w, e); break;
    case 8: dw_reduce_job<8>(a, i0, n, w, e); break;
    default: dw_reduce_job<9>(a, i0, n, w, e); break;
  }
}
#endif

}  // namespace mlp
}  // namespace nerf

#ifndef NERF_MLP_DEVICE_ONLY
// ======================================================================================
// C-ABI
// ======================================================================================
using namespace nerf;
using namespace nerf::mlp;

template <class P> static constexpr size_t fwd_lds_bytes() { return (size_t)NSLOT * SLOT_CAP * 1024; }
template <class P> static constexpr size_t dx_lds_bytes() { return (size_t)NSLOT * SLOT_CAP * 1024; }
template <class P> static constexpr size_t dw_lds_bytes() { return (size_t)dw_nbuf<P>() * DW_SLOTS * P::CH * 1024; }

template <class K>
static void allow_lds(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <class P, bool STORE, bool DENSITY, bool HALF = false>
static void launch_fwd(const FwdArgs& a, hipStream_t stream) {
  static const bool lds_ok = (allow_lds(fwd_kernel<P, STORE, DENSITY, false, HALF>, fwd_lds_bytes<P>()), true);
  (void)lds_ok;
  const int spb = samples_per_block<P>();
  dim3 grid((unsigned)(STORE ? a.nblk * 32 / spb : (a.M + spb - 1) / spb));
  hipLaunchKernelGGL((fwd_kernel<P, STORE, DENSITY, false, HALF>), grid, dim3(P::WAVES * 64), fwd_lds_bytes<P>(),
                     stream, a);
}

// persistent inference forward: one wave of workgroups (every CU x its resident workgroups),
// fewer when M_cap needs fewer blocks
template <class P>
static void launch_fwd_persist(const FwdArgs& a, hipStream_t stream) {
  auto kern = fwd_kernel<P, false, false, true>;
  static const int resident = [&] {
    allow_lds(kern, fwd_lds_bytes<P>());
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)kern, P::WAVES * 64, fwd_lds_bytes<P>()) !=
            hipSuccess || per <= 0)
      per = 1;
    return cus * per;
  }();
  const int64_t spb = samples_per_block<P>(), need = (a.M_cap + spb - 1) / spb;
  dim3 grid((unsigned)(need < resident ? need : resident));
  hipLaunchKernelGGL(kern, grid, dim3(P::WAVES * 64), fwd_lds_bytes<P>(), stream, a);
}

template <class P>
static void launch_dx(const DxArgs& x, int64_t ldm, hipStream_t stream) {
  static const bool lds_ok = (allow_lds(dx_kernel<P>, dx_lds_bytes<P>()), true);
  (void)lds_ok;
  hipLaunchKernelGGL((dx_kernel<P>), dim3((unsigned)(ldm / samples_per_block<P>())), dim3(P::WAVES * 64),
                     dx_lds_bytes<P>(), stream, x);
}

template <class P>
static void launch_fwd_any(const FwdArgs& a, bool store, bool density, hipStream_t stream) {
  if (store) launch_fwd<P, true, false>(a, stream);
  else if (density) launch_fwd<P, false, true>(a, stream);
  else launch_fwd<P, false, false>(a, stream);
}

// Every kernel launch of one precision, instantiated in that precision's translation unit
// (mlp.hip compiled with -DNERF_MLP_PREC=0 fp32 / 1 bf16 / 2 bf16x3, csrc/Makefile); the C-ABI
// unit (no NERF_MLP_PREC) only declares them, so the three precisions compile in parallel.
namespace nerf {
namespace mlp {
// the pack plan of (P, dir) on the device that holds the parameters: built on first use (one launch, then a
// stream sync), kept for the process; null if it cannot be allocated, or while the stream is being captured
// (the build syncs), and the caller falls back to pack_kernel.  The device comes from the parameter pointer,
// not the current device (a net on cuda:1 packed while cuda:0 is current), and the build runs under a device
// guard on that device.  (round 6)
static_assert(NET_PARAMS < (1 << 24), "a plan entry holds a 24-bit parameter offset");
// the packed-weight layout of a policy's forward: 32-row units (0), or the 16-row units of PBF3W (2)
template <class P> static constexpr int fwd_layout() { return wide_kind<P>() ? 2 : 0; }
// ... and of its dX: 32-row units (1), or the 16-row units of PF32W / PBF3W (3)
template <class P> static constexpr int bwd_layout() { return wide_kind<P>() ? 3 : 1; }
template <class P, class F> static void with_layout(int dir, F&& f) {  // f(integral_constant<layout>)
  if (dir == 1) {
    f(std::integral_constant<int, bwd_layout<P>()>{});
  } else {
    f(std::integral_constant<int, fwd_layout<P>()>{});
  }
}
template <class P>
static const uint32_t* pack_plan(int dir, const void* params, hipStream_t stream) {
  static std::mutex mu;
  static uint32_t* plans[64][2] = {};
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, params) != hipSuccess || at.device < 0 || at.device >= 64) return nullptr;
  const int dev = at.device;
  std::lock_guard<std::mutex> lock(mu);
  uint32_t*& plan = plans[dev][dir];
  if (!plan) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || (cur != dev && hipSetDevice(dev) != hipSuccess)) return nullptr;
    const int64_t n = total_chunks(P::CH, dir == 0 ? fwd_layout<P>() : bwd_layout<P>()) * 64;
    uint32_t* p = nullptr;
    bool ok = hipMalloc(&p, (size_t)n * P::E * sizeof(uint32_t)) == hipSuccess;
    if (ok) {
      dim3 grid((unsigned)((n + 255) / 256));
      with_layout<P>(dir, [&](auto lay) {
        constexpr int D = decltype(lay)::value;
        hipLaunchKernelGGL((pack_plan_kernel<P, D>), grid, dim3(256), 0, stream, unit_offsets<P::CH, D>(), p);
      });
      ok = hipStreamSynchronize(stream) == hipSuccess;
      if (!ok) (void)hipFree(p);
    }
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return nullptr;
    plan = p;
  }
  return plan;
}
template <class P>
void mlp_pack_impl(const ParamPtrs& prm, int dir, char* dst, hipStream_t stream) {
  const int64_t n = total_chunks(P::CH, dir == 0 ? fwd_layout<P>() : bwd_layout<P>()) * 64;
  dim3 grid((unsigned)((n + 255) / 256));
  // the 24 parameters back to back (FusedAdam's flat buffer): the plan gather (NERF_PACK_PLAN=0: always
  // the direct pack, for A/B timing)
  const char* env = getenv("NERF_PACK_PLAN");
  bool flat = !(env && env[0] == '0');
  for (int k = 1; k < NPARAM; ++k) flat = flat && prm.p[k] == prm.p[0] + param_offset(k);
  if (flat) {
    if (const uint32_t* plan = pack_plan<P>(dir, prm.p[0], stream)) {
      hipLaunchKernelGGL((pack_gather_kernel<P>), grid, dim3(256), 0, stream, prm.p[0], plan, dst, n);
      return;
    }
  }
  with_layout<P>(dir, [&](auto lay) {
    constexpr int D = decltype(lay)::value;
    hipLaunchKernelGGL((pack_kernel<P, D>), grid, dim3(256), 0, stream, prm, unit_offsets<P::CH, D>(), dst);
  });
}
template <class P>
void mlp_fwd_train_impl(const FwdArgs& a, hipStream_t stream) {
  launch_fwd<P, true, false>(a, stream);
}
// The bf16x3 forward (training, bf16x3f training with bf16 stores, inference, density, persistent): the wide
// 16x16x32 kernel (PBF3W, round 6) or, with -DNERF_BF3_WIDE=0, the 32x32x16 one (PBF3) for A/B builds.  The
// bf16x3 backward (dX / dW, and its W^T pack) is PBF3's either way: both forwards write the same stores.
#ifndef NERF_BF3_WIDE
#define NERF_BF3_WIDE 1
#endif
using PBF3F = std::conditional_t<NERF_BF3_WIDE != 0, PBF3W, PBF3>;
// The fp32 TRAINING forward: PF32's, or with -DNERF_F32_WIDE=1 the wide 16x16x4 kernel (PF32W, round 6; the
// inference forwards -- renders, the march, the bake -- stay PF32 either way: another summation order moves the
// few ill-conditioned CDF bins of the full-frame fixtures).  The fp32 forward pack then holds both
// layouts, PF32's units first (nerf_mlp_packed_bytes), and the training forward reads the second.  Not the
// default (profiles/r6/f32w_*.json): 4.9 % faster (4.863 -> 4.625 ms per 524,288 samples), deterministic, masks
// equal to its activations' non-zeros, raw within 2.7e-7 of PF32's -- but its summation order flips the ReLU
// branch of a few near-zero pre-activations that PF32's order and the reference's agree on, and the 4,096-ray
// fine-net L0 bias gradient then sits 9.4e-4 (of the tensor's largest) from the reference's against the fp32
// contract's 1e-4 (PF32: 5.5e-5; tests/test_gpu_trained.py::test_loss_gradients_fp32).
#ifndef NERF_F32_WIDE
#define NERF_F32_WIDE 0
#endif
using PF32T = std::conditional_t<NERF_F32_WIDE != 0, PF32W, PF32>;
[[maybe_unused]] constexpr int64_t F32W_PACK_OFF = NERF_F32_WIDE ? total_chunks(PF32::CH, 0) * 1024 : 0;
// The dX of fp32 and bf16x3: the wide 16x16 kernels (DxWave16 over 16-row units, round 6) or, with
// -DNERF_F32_WIDE_DX=0 / -DNERF_BF3_WIDE_DX=0, the 32x32 ones; their W^T packs follow (bwd_layout).  The dZ they
// store is the same old-layout tile-block list either way (the dW is unchanged).
#ifndef NERF_F32_WIDE_DX
#define NERF_F32_WIDE_DX 1
#endif
#ifndef NERF_BF3_WIDE_DX
#define NERF_BF3_WIDE_DX 1
#endif
// (the bf16 dX stays the 32x32 kernel: the wide one, PBF16W, reads a 1 KiB weight chunk per single 16x16x32 MFMA --
// twice the LDS bytes per flop of the 32x32 kernel's, which already ran two waves per SIMD -- and measured slower,
// bf16 dX 0.596 -> 0.747 ms, bf16x3f's 0.564 -> 0.724, profiles/r6/wide_dx_bf16_ab.json; -DNERF_BF16_WIDE_DX=1)
#ifndef NERF_BF16_WIDE_DX
#define NERF_BF16_WIDE_DX 0
#endif
using PF32X = std::conditional_t<NERF_F32_WIDE_DX != 0, PF32W, PF32>;
using PBF16X = std::conditional_t<NERF_BF16_WIDE_DX != 0, PBF16W, PBF16>;  // (the bf16 / bf16x3f dX)
using PBF3X = std::conditional_t<NERF_BF3_WIDE_DX != 0, PBF3W, PBF3>;
// bf16x3 forward, bf16 (hi-half) stores for the bf16 backward
void mlp_fwd_train_half_impl(const FwdArgs& a, hipStream_t stream);
#if defined(NERF_MLP_PREC) && NERF_MLP_PREC == 2 && (!defined(NERF_MLP_PART) || NERF_MLP_PART == 4)
void mlp_fwd_train_half_impl(const FwdArgs& a, hipStream_t stream) { launch_fwd<PBF3F, true, false, true>(a, stream); }
#endif
// the three inference forwards, one translation unit each (parts 1, 5, 6)
template <class P>
void mlp_fwd_plain_impl(const FwdArgs& a, hipStream_t stream) { launch_fwd<P, false, false>(a, stream); }
template <class P>
void mlp_fwd_density_impl(const FwdArgs& a, hipStream_t stream) { launch_fwd<P, false, true>(a, stream); }
template <class P>
void mlp_fwd_persist_impl(const FwdArgs& a, hipStream_t stream) { launch_fwd_persist<P>(a, stream); }
template <class P>
void mlp_fwd_infer_impl(const FwdArgs& a, bool density, hipStream_t stream) {
  if (a.M_dev) mlp_fwd_persist_impl<P>(a, stream);
  else if (density) mlp_fwd_density_impl<P>(a, stream);
  else mlp_fwd_plain_impl<P>(a, stream);
}
template <class P>
void mlp_dx_impl(const DxArgs& x, int64_t ldm, hipStream_t stream) {
  launch_dx<P>(x, ldm, stream);
}
template <class P>
void mlp_dw_impl(const DwArgs& w, dim3 grid, hipStream_t stream) {
  allow_lds(dw_kernel<P>, dw_lds_bytes<P>());
  hipLaunchKernelGGL((dw_kernel<P>), grid, dim3(DW_WAVES * 64), dw_lds_bytes<P>(), stream, w);
}
// explicit instantiations, split further by part (-DNERF_MLP_PART: 0 training forward, 1 inference
// and density forwards, 2 dX + pack, 3 dW) so that no translation unit holds more than one or two
// of the large straight-line kernels
#define NERF_MLP_I_PACK(EXT, P) EXT template void mlp_pack_impl<P>(const ParamPtrs&, int, char*, hipStream_t);
#define NERF_MLP_I_FWDT(EXT, P) EXT template void mlp_fwd_train_impl<P>(const FwdArgs&, hipStream_t);
#define NERF_MLP_I_FWDI(EXT, P) EXT template void mlp_fwd_plain_impl<P>(const FwdArgs&, hipStream_t);
#define NERF_MLP_I_FWDD(EXT, P) EXT template void mlp_fwd_density_impl<P>(const FwdArgs&, hipStream_t);
#define NERF_MLP_I_FWDP(EXT, P) EXT template void mlp_fwd_persist_impl<P>(const FwdArgs&, hipStream_t);
#define NERF_MLP_I_DX(EXT, P) EXT template void mlp_dx_impl<P>(const DxArgs&, int64_t, hipStream_t);
#define NERF_MLP_I_DW(EXT, P) EXT template void mlp_dw_impl<P>(const DwArgs&, dim3, hipStream_t);
#define NERF_MLP_IMPLS(EXT, P) \
  NERF_MLP_I_PACK(EXT, P) NERF_MLP_I_FWDT(EXT, P) NERF_MLP_I_FWDI(EXT, P) NERF_MLP_I_FWDD(EXT, P) \
  NERF_MLP_I_FWDP(EXT, P) NERF_MLP_I_DX(EXT, P) NERF_MLP_I_DW(EXT, P)
#define NERF_MLP_FWDS(EXT, P) \
  NERF_MLP_I_FWDT(EXT, P) NERF_MLP_I_FWDI(EXT, P) NERF_MLP_I_FWDD(EXT, P) NERF_MLP_I_FWDP(EXT, P)
#if !defined(NERF_MLP_PREC)
NERF_MLP_IMPLS(extern, PF32)
NERF_MLP_I_FWDT(extern, PF32W)
NERF_MLP_I_PACK(extern, PF32W)
NERF_MLP_I_DX(extern, PF32W)
NERF_MLP_I_DX(extern, PBF3W)
NERF_MLP_I_DX(extern, PBF16W)
NERF_MLP_I_PACK(extern, PBF16W)
NERF_MLP_IMPLS(extern, PBF16)
NERF_MLP_I_PACK(extern, PBF3)  // bf16x3: the W^T pack, dX, dW (+ the forward pack when not wide)
NERF_MLP_I_DX(extern, PBF3)
NERF_MLP_I_DW(extern, PBF3)
NERF_MLP_FWDS(extern, PBF3F)
NERF_MLP_I_PACK(extern, PBF3W)
NERF_MLP_I_FWDI(extern, PBF6)  // bf16x6: the inference forward and its pack only
NERF_MLP_I_PACK(extern, PBF6)
#elif NERF_MLP_PREC == 3
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 1
NERF_MLP_I_FWDI(, PBF6)
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 2
NERF_MLP_I_PACK(, PBF6)
#endif
#else
#if NERF_MLP_PREC == 0
#define NERF_PP PF32
#elif NERF_MLP_PREC == 1
#define NERF_PP PBF16
#else
#define NERF_PP PBF3
#endif
#if NERF_MLP_PREC == 2
#define NERF_PP_FWD PBF3F  // (the bf16x3 forwards: PBF3W unless NERF_BF3_WIDE=0)
#else
#define NERF_PP_FWD NERF_PP
#endif
#if NERF_MLP_PREC == 0
#define NERF_PP_FWDT PF32T  // (the fp32 training forward: PF32W unless NERF_F32_WIDE=0)
#else
#define NERF_PP_FWDT NERF_PP_FWD
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 0
NERF_MLP_I_FWDT(, NERF_PP_FWDT)
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 1
NERF_MLP_I_FWDI(, NERF_PP_FWD)
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 5
NERF_MLP_I_FWDD(, NERF_PP_FWD)
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 6
NERF_MLP_I_FWDP(, NERF_PP_FWD)
#endif
#if NERF_MLP_PREC == 0
#define NERF_PP_DX PF32X  // (the fp32 dX: PF32W unless NERF_F32_WIDE_DX=0)
#elif NERF_MLP_PREC == 2
#define NERF_PP_DX PBF3X  // (the bf16x3 dX: PBF3W unless NERF_BF3_WIDE_DX=0)
#elif NERF_MLP_PREC == 1
#define NERF_PP_DX PBF16X  // (the bf16 dX: PBF16W unless NERF_BF16_WIDE_DX=0)
#else
#define NERF_PP_DX NERF_PP
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 2
NERF_MLP_I_DX(, NERF_PP_DX)
NERF_MLP_I_PACK(, NERF_PP)
#if NERF_MLP_PREC == 2 && (NERF_BF3_WIDE || NERF_BF3_WIDE_DX)
NERF_MLP_I_PACK(, PBF3W)
#endif
#if NERF_MLP_PREC == 0 && (NERF_F32_WIDE || NERF_F32_WIDE_DX)
NERF_MLP_I_PACK(, PF32W)
#endif
#if NERF_MLP_PREC == 1 && NERF_BF16_WIDE_DX
NERF_MLP_I_PACK(, PBF16W)
#endif
#endif
#if !defined(NERF_MLP_PART) || NERF_MLP_PART == 3
NERF_MLP_I_DW(, NERF_PP)
#endif
#endif
}  // namespace mlp
}  // namespace nerf

#if !defined(NERF_MLP_PREC)

extern "C" {

int64_t nerf_mlp_net_params(void) { return NET_PARAMS; }
int64_t nerf_mlp_param_offset(int i) { return (i >= 0 && i <= NPARAM) ? param_offset(i) : -1; }

// dtype 3 (bf16x3f) = a bf16x3 forward (its forward pack) whose training stores are bf16, with
// the bf16 backward (its W^T pack, bf16 dZ): every function below maps it to its part
static int fwd_prec(int dtype) { return dtype == 3 ? 2 : dtype; }
static int bwd_prec(int dtype) { return dtype == 3 ? 1 : dtype; }
static int store_prec(int dtype) { return dtype == 3 ? 1 : dtype; }
// dtype 4 (bf16x6) is an inference forward only: its forward pack and nerf_mlp_fwd without flags
static bool train_dtype(int dtype) { return dtype >= 0 && dtype <= 3; }

int64_t nerf_mlp_packed_bytes(int dtype, int dir) {
  if (dtype == 4) return dir == 0 ? total_chunks(PBF6::CH, 0) * 1024 : -1;
  if (!train_dtype(dtype) || (dir != 0 && dir != 1)) return -1;
  const int p = dir == 0 ? fwd_prec(dtype) : bwd_prec(dtype);
  if (p == 2 && dir == 0) return total_chunks(PBF3F::CH, fwd_layout<PBF3F>()) * 1024;  // (the wide bf16x3 forward)
  if (p == 0 && dir == 0 && NERF_F32_WIDE)  // PF32's units, then PF32W's (the training forward)
    return F32W_PACK_OFF + total_chunks(PF32W::CH, fwd_layout<PF32W>()) * 1024;
  if (p == 0 && dir == 1) return total_chunks(PF32X::CH, bwd_layout<PF32X>()) * 1024;  // (the fp32 dX)
  if (p == 2 && dir == 1) return total_chunks(PBF3X::CH, bwd_layout<PBF3X>()) * 1024;  // (the bf16x3 dX)
  if (p == 1 && dir == 1) return total_chunks(PBF16X::CH, bwd_layout<PBF16X>()) * 1024;  // (the bf16 dX)
  return total_chunks(p == 1 ? PBF16::CH : PF32::CH, dir) * 1024;  // bf16x3: CH 4 as fp32
}

int64_t nerf_mlp_padded_samples(int64_t M) { return (M + M_ALIGN - 1) / M_ALIGN * M_ALIGN; }
int64_t nerf_mlp_act_bytes(int dtype, int64_t M) {
  if (dtype < 0 || dtype > 3 || M < 0) return -1;
  return (int64_t)A_ROWS * nerf_mlp_padded_samples(M) * (store_prec(dtype) == 1 ? 2 : 4);
}
int64_t nerf_mlp_dz_bytes(int dtype, int64_t M) {
  if (dtype < 0 || dtype > 3 || M < 0) return -1;
  return (int64_t)Z_ROWS * nerf_mlp_padded_samples(M) * (store_prec(dtype) == 1 ? 2 : 4);
}
int64_t nerf_mlp_mask_bytes(int64_t M) { return nerf_mlp_padded_samples(M) / 32 * MASK_GROUPS * 64 * 16; }

int nerf_mlp_pack(const float* const* params, int dtype, void* packed_fwd, void* packed_bwd, hipStream_t stream) {
  NERF_REQUIRE(params != nullptr, "nerf_mlp_pack: params is null");
  NERF_REQUIRE(dtype >= 0 && dtype <= 4,
               "nerf_mlp_pack: dtype must be 0 (f32), 1 (bf16), 2 (bf16x3), 3 (bf16x3f) or 4 (bf16x6), got %d", dtype);
  NERF_REQUIRE(dtype != 4 || packed_bwd == nullptr, "nerf_mlp_pack: dtype 4 (bf16x6) has no backward pack");
  ParamPtrs prm;
  for (int i = 0; i < NPARAM; ++i) {
    NERF_REQUIRE(params[i] != nullptr, "nerf_mlp_pack: params[%d] is null", i);
    prm.p[i] = params[i];
  }
  for (int dir = 0; dir < 2; ++dir) {
    void* dst = dir == 0 ? packed_fwd : packed_bwd;
    if (!dst) continue;
    const int p = dir == 0 ? fwd_prec(dtype) : bwd_prec(dtype);
    if (p == 4) mlp_pack_impl<PBF6>(prm, dir, (char*)dst, stream);
    else if (p == 0 && dir == 1) mlp_pack_impl<PF32X>(prm, dir, (char*)dst, stream);
    else if (p == 0) {
      mlp_pack_impl<PF32>(prm, dir, (char*)dst, stream);
      if (dir == 0 && NERF_F32_WIDE) mlp_pack_impl<PF32T>(prm, dir, (char*)dst + F32W_PACK_OFF, stream);
    }
    else if (p == 1 && dir == 1) mlp_pack_impl<PBF16X>(prm, dir, (char*)dst, stream);
    else if (p == 1) mlp_pack_impl<PBF16>(prm, dir, (char*)dst, stream);
    else if (dir == 0) mlp_pack_impl<PBF3F>(prm, dir, (char*)dst, stream);
    else mlp_pack_impl<PBF3X>(prm, dir, (char*)dst, stream);
    if (int e = check_launch("nerf_mlp_pack")) return e;
  }
  return 0;
}

// flags: bit0 = store activations + masks for backward, bit1 = density only
int nerf_mlp_fwd(const void* packed_fwd, int dtype, const float* pts, const float* viewdirs, int samples_per_dir,
                 const int32_t* dir_index, int64_t M, int flags, float* raw, void* act, uint16_t* masks,
                 hipStream_t stream) {
  NERF_REQUIRE(dtype >= 0 && dtype <= 4, "nerf_mlp_fwd: bad dtype %d", dtype);
  NERF_REQUIRE(dtype != 4 || flags == 0, "nerf_mlp_fwd: dtype 4 (bf16x6) is an inference forward only (flags 0)");
  NERF_REQUIRE(M >= 0, "nerf_mlp_fwd: M < 0");
  if (M == 0) return 0;
  const bool store = flags & 1, density = flags & 2;
  NERF_REQUIRE(packed_fwd && pts && raw, "nerf_mlp_fwd: null pointer");
  NERF_REQUIRE(density || viewdirs, "nerf_mlp_fwd: viewdirs required unless density-only");
  NERF_REQUIRE(density || dir_index || samples_per_dir > 0, "nerf_mlp_fwd: samples_per_dir must be > 0");
  NERF_REQUIRE(!store || (act && masks), "nerf_mlp_fwd: store requires act and masks");
  NERF_REQUIRE(!(store && density), "nerf_mlp_fwd: store and density-only are exclusive");
  FwdArgs a{(const char*)packed_fwd, pts, viewdirs, dir_index, samples_per_dir, M,
            nerf_mlp_padded_samples(M) / 32, raw, act, masks};
  if (store) {
    if (dtype == 0) {
      a.wpack += F32W_PACK_OFF;  // (the PF32W units of the fp32 pack)
      mlp_fwd_train_impl<PF32T>(a, stream);
    }
    else if (dtype == 1) mlp_fwd_train_impl<PBF16>(a, stream);
    else if (dtype == 2) mlp_fwd_train_impl<PBF3F>(a, stream);
    else mlp_fwd_train_half_impl(a, stream);
  } else {
    if (dtype == 4) mlp_fwd_plain_impl<PBF6>(a, stream);
    else if (dtype == 0) mlp_fwd_infer_impl<PF32>(a, density, stream);
    else if (dtype == 1) mlp_fwd_infer_impl<PBF16>(a, density, stream);
    else mlp_fwd_infer_impl<PBF3F>(a, density, stream);
  }
  return check_launch("nerf_mlp_fwd");
}

// inference forward whose sample count is on the device (min(*M_dev, M_cap)): no host sync sizes
// the launch (the grid march's rounds)
int nerf_mlp_fwd_count(const void* packed_fwd, int dtype, const float* pts, const float* viewdirs, int samples_per_dir,
                       const int32_t* dir_index, const int32_t* M_dev, int64_t M_cap, float* raw, hipStream_t stream) {
  NERF_REQUIRE(dtype >= 0 && dtype <= 3, "nerf_mlp_fwd_count: bad dtype %d", dtype);
  NERF_REQUIRE(M_cap >= 0, "nerf_mlp_fwd_count: M_cap < 0");
  if (M_cap == 0) return 0;
  NERF_REQUIRE(packed_fwd && pts && raw && viewdirs && M_dev, "nerf_mlp_fwd_count: null pointer");
  NERF_REQUIRE(dir_index || samples_per_dir > 0, "nerf_mlp_fwd_count: samples_per_dir must be > 0");
  FwdArgs a{(const char*)packed_fwd, pts, viewdirs, dir_index, samples_per_dir, M_cap, 0, raw, nullptr, nullptr,
            M_dev, M_cap};
  if (dtype == 0) mlp_fwd_infer_impl<PF32>(a, false, stream);
  else if (dtype == 1) mlp_fwd_infer_impl<PBF16>(a, false, stream);
  else mlp_fwd_infer_impl<PBF3F>(a, false, stream);
  return check_launch("nerf_mlp_fwd_count");
}

// work items of the dW launch: at most one per CU (a single wave of workgroups that ends
// together), split across the 10 jobs in proportion to the bytes each reads, at least one
// and at most one per block per job
static int cu_count() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || n <= 0)
    n = 256;
  return n;
}
// cost (SIMD cycles) of one 32-sample block of job j.  bf16 dW is HBM-bound and its 4-deep
// ring hides the fetch latency: the tile-blocks streamed.  fp32 dW: the busiest wave pair's
// MFMAs (2 waves x 16 K steps x (k-tiles, + the alpha row for feature/alpha, 9 for the view
// layer's waves 0..3) x 64 cycles), or -- for the light L0 job, behind a 2-deep ring -- the
// block's fetch: its latency + its bytes at a CU's share of HBM (~25 GB/s, 393 cycles per
// 4 KiB tile).
#ifndef NERF_DW_BALANCE_MFMA
#define NERF_DW_BALANCE_MFMA 1
#endif
#ifndef NERF_DW_LAT_CYCLES
#define NERF_DW_LAT_CYCLES 4000
#endif
// fp32: two items per CU (measured -2.5 % over one: the tail of the last items is shorter);
// bf16: one (every extra item re-adds its partial dW with atomics)
#ifndef NERF_DW_ITEMS_PER_CU
#define NERF_DW_ITEMS_PER_CU 2
#endif
// fp32 (NERF_DW_COST_TABLE 1, default): each job's measured time with the whole chip to itself
// (diagnostic build -DNERF_DW_DIAG, NERF_DW_ONLY_JOB=j, tools/gpu_dw_jobs.sh; per mille of the L1
// job) replaces the model below, which under-priced L5 (measured 1.42x L1, modelled 1.25x) and
// over-priced the view job (0.79x, modelled 1.13x) and L0: dW 4.94 -> 4.72 ms at 524k samples
#ifndef NERF_DW_COST_TABLE
#define NERF_DW_COST_TABLE 1
#endif
#ifndef NERF_DW_COST_TABLE_BF
#define NERF_DW_COST_TABLE_BF 1
#endif
static int64_t dw_job_cost(int dtype, int j) {
  static constexpr int64_t MEASURED[3][NDWJOB] = {{332, 1000, 1014, 1021, 1018, 1418, 1024, 1012, 1131, 792},
                                                  {560, 1000, 1009, 999, 1009, 1733, 1001, 1012, 1117, 1072},  // (unused)
                                                  {552, 1000, 1011, 1004, 1004, 1465, 1003, 1007, 1144, 1044}};
  if (dtype == 0 && NERF_DW_COST_TABLE) return MEASURED[0][j] * 16;
  // bf16x3 too (2.005 -> 1.943 ms); not bf16, whose jobs all stream HBM at once: its solo timings
  // (L5 1.73x L1) misprice the shared-bandwidth run (0.914 -> 0.949 ms), the tile count does not
  if (dtype == 2 && NERF_DW_COST_TABLE_BF) return MEASURED[2][j];
  if (dtype != 0 || !NERF_DW_BALANCE_MFMA) return dw_job_tiles(j);
  const int64_t mfma = 2 * 16 * (j < 8 ? gemm_k_tiles(j) : 9) * 64;
  const int64_t fetch = NERF_DW_LAT_CYCLES + 393 * (int64_t)dw_job_tiles(j);
  return mfma > fetch ? mfma : fetch;
}
constexpr int64_t DW_MIN_BLOCKS = 8;  // 32-sample blocks per dW work item, at least
static void dw_items(int dtype, int64_t nblk, int item_off[NDWJOB + 1], int job_of[NDWJOB]) {
  static const int cus = cu_count();
  const int target = cus * (dtype == 0 ? NERF_DW_ITEMS_PER_CU : 1);
  int n[NDWJOB];
  int64_t cost = 0;
  for (int j = 0; j < NDWJOB; ++j) cost += dw_job_cost(dtype, j);
  // a small launch (a 64-ray chunk: 128 blocks) gets few items, each of >= DW_MIN_BLOCKS blocks:
  // every item adds a 364 KB partial-sum slice that the ordered reduce reads back
  const int64_t max_items = nblk / DW_MIN_BLOCKS > 1 ? nblk / DW_MIN_BLOCKS : 1;
  int total = 0;
  for (int j = 0; j < NDWJOB; ++j) {
    int64_t k = target * (int64_t)dw_job_cost(dtype, j) / cost;
    n[j] = (int)(k < 1 ? 1 : k > max_items ? max_items : k);
    total += n[j];
  }
  // the remaining CUs go, one at a time, to the job whose items are the longest
  while (total < target) {
    int best = -1;
    double worst = 0.0;  // (worst = 0 only before the first candidate)
    for (int j = 0; j < NDWJOB; ++j) {
      if (n[j] >= max_items) continue;
      const double per = (double)dw_job_cost(dtype, j) / n[j];
      if (per > worst) worst = per, best = j;
    }
    if (best < 0) break;
    ++n[best];
    ++total;
  }
  // longest items first: with more items than CUs, the short ones fill the tail
  for (int j = 0; j < NDWJOB; ++j) job_of[j] = j;
  for (int a = 0; a < NDWJOB; ++a)
    for (int b = a + 1; b < NDWJOB; ++b)
      if ((double)dw_job_cost(dtype, job_of[b]) / n[job_of[b]] > (double)dw_job_cost(dtype, job_of[a]) / n[job_of[a]]) {
        const int t = job_of[a];
        job_of[a] = job_of[b];
        job_of[b] = t;
      }
  item_off[0] = 0;
  for (int s = 0; s < NDWJOB; ++s) item_off[s + 1] = item_off[s] + n[job_of[s]];
#ifdef NERF_DW_DIAG
  // (diagnostic build only) NERF_DW_ONLY_JOB=j: every item to job j, the others skipped
  if (const char* e = getenv("NERF_DW_ONLY_JOB")) {
    const int jj = atoi(e);
    job_of[0] = jj;  // segments 1.. are empty
    for (int s = 1; s <= NDWJOB; ++s) item_off[s] = target;
  }
#endif
}
int64_t nerf_mlp_dw_items(int dtype, int64_t M) {
  if (dtype < 0 || dtype > 3 || M < 0) return -1;
  int off[NDWJOB + 1], job[NDWJOB];
  dw_items(bwd_prec(dtype), nerf_mlp_padded_samples(M) / 32, off, job);
  return off[NDWJOB];
}

// dX chain only: dz (per-layer output gradients, fragment-native tiles) from d_raw + masks
int nerf_mlp_bwd_dx(const void* packed_bwd, int dtype, const float* d_raw, int64_t M, const uint16_t* masks, void* dz,
                    hipStream_t stream) {
  NERF_REQUIRE(dtype >= 0 && dtype <= 3, "nerf_mlp_bwd_dx: bad dtype %d", dtype);
  dtype = bwd_prec(dtype);
  NERF_REQUIRE(M >= 0, "nerf_mlp_bwd_dx: M < 0");
  if (M == 0) return 0;
  NERF_REQUIRE(packed_bwd && d_raw && masks && dz, "nerf_mlp_bwd_dx: null pointer");
  const int64_t ldm = nerf_mlp_padded_samples(M);
  DxArgs x{(const char*)packed_bwd, d_raw, M, ldm / 32, masks, dz};
  if (dtype == 0) mlp_dx_impl<PF32X>(x, ldm, stream);
  else if (dtype == 1) mlp_dx_impl<PBF16X>(x, ldm, stream);
  else mlp_dx_impl<PBF3X>(x, ldm, stream);
  return check_launch("nerf_mlp_bwd_dx");
}

int64_t nerf_mlp_dw_workspace_bytes(int dtype, int64_t M) {
  const int64_t items = nerf_mlp_dw_items(dtype, M);
  return items < 0 ? -1 : items * (int64_t)DW_PITEM * 4;
}

// dW/db only: grad += dz . act^T (grad must be zeroed or hold a running sum).  workspace (nullable,
// nerf_mlp_dw_workspace_bytes): per-item partial sums reduced in a fixed order -- bit-reproducible;
// null: fp32 atomics.
int nerf_mlp_bwd_dw_ws(int dtype, int64_t M, const void* act, const void* dz, float* grad, void* workspace,
                       hipStream_t stream) {
  NERF_REQUIRE(dtype >= 0 && dtype <= 3, "nerf_mlp_bwd_dw: bad dtype %d", dtype);
  dtype = bwd_prec(dtype);
  NERF_REQUIRE(M >= 0, "nerf_mlp_bwd_dw: M < 0");
  if (M == 0) return 0;
  NERF_REQUIRE(act && dz && grad, "nerf_mlp_bwd_dw: null pointer");
  const int64_t nblk = nerf_mlp_padded_samples(M) / 32;
  DwArgs w{dz, act, nblk, grad, {}, {}, (float*)workspace};
  dw_items(dtype, nblk, w.item_off, w.job_of);
  dim3 grid((unsigned)w.item_off[NDWJOB]);
  if (dtype == 0) mlp_dw_impl<PF32>(w, grid, stream);
  else if (dtype == 1) mlp_dw_impl<PBF16>(w, grid, stream);
  else mlp_dw_impl<PBF3>(w, grid, stream);
  if (int e = check_launch("nerf_mlp_bwd_dw")) return e;
  if (workspace) {
    DwReduceArgs r{(const float*)workspace, grad, {}, {}};
    for (int k = 0; k <= NDWJOB; ++k) r.item_off[k] = w.item_off[k];
    for (int k = 0; k < NDWJOB; ++k) r.job_of[k] = w.job_of[k];
    const int64_t per = (int64_t)DW_WAVES * DW_PWAVE;
    hipLaunchKernelGGL(dw_reduce_kernel, dim3((unsigned)((per + 255) / 256), NDWJOB), dim3(256), 0, stream, r);
    return check_launch("nerf_mlp_bwd_dw_reduce");
  }
  return 0;
}
int nerf_mlp_bwd_dw(int dtype, int64_t M, const void* act, const void* dz, float* grad, hipStream_t stream) {
  return nerf_mlp_bwd_dw_ws(dtype, M, act, dz, grad, nullptr, stream);
}

int nerf_mlp_bwd(const void* packed_bwd, int dtype, const float* d_raw, int64_t M, const void* act,
                 const uint16_t* masks, void* dz, float* grad, hipStream_t stream) {
  if (int e = nerf_mlp_bwd_dx(packed_bwd, dtype, d_raw, M, masks, dz, stream)) return e;
  return nerf_mlp_bwd_dw(dtype, M, act, dz, grad, stream);
}

}  // extern "C"
#endif  // !NERF_MLP_PREC
#endif  // NERF_MLP_DEVICE_ONLY

// ------------------------------------------------------------------------------------
// Knob policy (round 6).  Schedule knobs -- NERF_FINISH_PARTS_*, NERF_FINISH_DELAY, NERF_PREFETCH_*,
// NERF_DMA_SPREAD_*, NERF_GROUP_ACROSS -- may take any value: every placement they produce is proven at compile
// time (FinishSchedule's static_assert in FwdWave / FwdWave16 / DxWave; the hand-off vmcnt counts are computed
// from the same tables and tools/asm_check.py checks them on the emitted code).  NERF_BF3_WIDE and NERF_*_WIDE_DX
// select between verified kernels (below).  NERF_DIAG_* are diagnostic builds only (results meaningless).  Every other tuning
// knob is pinned to the value the tests verified: building another value fails here.
// ------------------------------------------------------------------------------------
#define NERF_PINNED(K, V) static_assert((K) == (V), #K ": only the verified value " #V " is allowed (mlp.hip knob policy)");
NERF_PINNED(NERF_PACKED_MASK, 1)
NERF_PINNED(NERF_DMA_LEAN, 1)
NERF_PINNED(NERF_KEEP_PE_BF3, 1)
NERF_PINNED(NERF_DW_NBUF_BF16, 4)
NERF_PINNED(NERF_DW_SWZ_F32, 1)
NERF_PINNED(NERF_DW_F32_PIPE, 1)
NERF_PINNED(NERF_DW_FETCH_STEP, 1)
NERF_PINNED(NERF_DW_FETCH_SPLIT, 4)
NERF_PINNED(NERF_DW_DMA_NT, 1)
#if defined(NERF_DW_BALANCE_MFMA)
NERF_PINNED(NERF_DW_BALANCE_MFMA, 1)
NERF_PINNED(NERF_DW_LAT_CYCLES, 4000)
NERF_PINNED(NERF_DW_ITEMS_PER_CU, 2)
NERF_PINNED(NERF_DW_COST_TABLE, 1)
NERF_PINNED(NERF_DW_COST_TABLE_BF, 1)
#endif
#if defined(NERF_BF3_WIDE)
static_assert(NERF_BF3_WIDE == 0 || NERF_BF3_WIDE == 1, "NERF_BF3_WIDE: 0 (32x32 bf16x3 forward) or 1 (wide)");
// (the other kernel selectors: NERF_F32_WIDE -- the wide fp32 training forward, opt-in, off the fp32 gradient
// contract; NERF_F32_WIDE_DX / NERF_BF3_WIDE_DX -- the wide dX, on; NERF_BF16_WIDE_DX -- the wide bf16 dX, opt-in,
// slower; each 0 or 1, every one of the kernels they select compiles under FinishSchedule and tools/asm_check.py)
static_assert((NERF_F32_WIDE == 0 || NERF_F32_WIDE == 1) && (NERF_F32_WIDE_DX == 0 || NERF_F32_WIDE_DX == 1) &&
                  (NERF_BF3_WIDE_DX == 0 || NERF_BF3_WIDE_DX == 1) && (NERF_BF16_WIDE_DX == 0 || NERF_BF16_WIDE_DX == 1),
              "NERF_*_WIDE*: 0 or 1");
#endif
#undef NERF_PINNED
