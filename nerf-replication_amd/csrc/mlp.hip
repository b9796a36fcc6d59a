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

namespace nerf {
namespace mlp {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// ------------------------------------------------------------------------------------
// precision policies
// ------------------------------------------------------------------------------------
struct PF32 {
  static constexpr int CH = 4;     // 1 KiB chunks per 32-feature input tile
  static constexpr int E = 4;      // elements per lane per chunk
  static constexpr int WAVES = 4;  // one wave per SIMD (<= 512 VGPR+AGPR)
  static constexpr int ESIZE = 4;
  static constexpr int SPL = 4;    // samples per 16-B lane load (dW GEMM)
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
  static __device__ __forceinline__ float get(const Tile& t, int rho) { return t.v[rho]; }
  static __device__ __forceinline__ Store cvt(float x) { return x; }
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
};

struct PBF16 {
  static constexpr int CH = 2;
  static constexpr int E = 8;
  static constexpr int WAVES = 8;  // two waves per SIMD (<= 256 VGPR)
  static constexpr int ESIZE = 2;
  static constexpr int SPL = 8;
  using Store = __bf16;
  struct Tile { bf16x8 b[2]; };
  static __device__ __forceinline__ f32x16 mma(uint4 a, const Tile& b, int c, f32x16 acc) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), b.b[c], acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void set(Tile& t, int rho, float x) { t.b[rho >> 3][rho & 7] = (__bf16)x; }
  static __device__ __forceinline__ float get(const Tile& t, int rho) { return (float)t.b[rho >> 3][rho & 7]; }
  static __device__ __forceinline__ Store cvt(float x) { return (__bf16)x; }
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
};

template <class P> __host__ __device__ constexpr int samples_per_block() { return P::WAVES * 32; }
constexpr int M_ALIGN = 256;  // activation stores are padded to this many samples

// ------------------------------------------------------------------------------------
// packed-weight layout (1 KiB chunks, lane-linear: chunk[lane][16 B])
//   forward unit u: fwd_unit_tiles(u) * CH weight chunks, then 1 bias chunk (32 fp32)
//   backward unit u: bwd_unit_tiles(u) * CH weight chunks
// ------------------------------------------------------------------------------------
__host__ __device__ constexpr int fwd_unit_chunks(int u, int ch) { return fwd_unit_tiles(u) * ch + 1; }
__host__ __device__ constexpr int fwd_unit_chunk_off(int u, int ch) { return fwd_unit_tile_off(u) * ch + u; }
__host__ __device__ constexpr int bwd_unit_chunks(int u, int ch) { return bwd_unit_tiles(u) * ch; }
__host__ __device__ constexpr int bwd_unit_chunk_off(int u, int ch) { return bwd_unit_tile_off(u) * ch; }
__host__ __device__ constexpr int64_t total_chunks(int ch, int dir) {
  return dir == 0 ? (int64_t)FWD_TILES * ch + NUNIT_FWD : (int64_t)BWD_TILES * ch;
}

struct ParamPtrs { const float* p[NPARAM]; };

// one thread per 16-B lane slot of one chunk
template <class P, int DIR>
__global__ void pack_kernel(ParamPtrs prm, char* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total_chunks(P::CH, DIR) * 64) return;
  const int lane = (int)(i & 63);
  const int chunk = (int)(i >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int nunit = DIR == 0 ? NUNIT_FWD : NUNIT_BWD;
  int u = 0;
  while (u + 1 < nunit &&
         (DIR == 0 ? fwd_unit_chunk_off(u + 1, P::CH) : bwd_unit_chunk_off(u + 1, P::CH)) <= chunk)
    ++u;
  const int within = chunk - (DIR == 0 ? fwd_unit_chunk_off(u, P::CH) : bwd_unit_chunk_off(u, P::CH));
  char* dst = out + i * 16;
  if (DIR == 0 && within == fwd_unit_tiles(u) * P::CH) {
    // bias chunk: lanes 0..7 hold the 32 biases of the unit's output rows, rest zero
    const int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
    const int wp = fwd_out_weight(L, n);
    float* d = (float*)dst;
    for (int e = 0; e < 4; ++e) {
      const int row = lane * 4 + e;
      d[e] = (lane < 8 && row < fwd_out_valid(L, n)) ? prm.p[wp + 1][fwd_out_row0(L, n) + row] : 0.f;
    }
    return;
  }
  const int t = within / P::CH, c = within % P::CH;
  typename P::Store vals[P::E];
#pragma unroll
  for (int e = 0; e < P::E; ++e) {
    const int rho = c * P::E + e;
    const int ar = acc_row(rho, h);
    float v = 0.f;
    if (DIR == 0) {
      const int L = fwd_unit_layer(u), n = u - fwd_unit_first(L);
      const int wp = fwd_out_weight(L, n);
      const int row = fwd_out_row0(L, n) + r, col = fwd_in_colbase(L, t) + ar;
      if (r < fwd_out_valid(L, n) && ar < fwd_in_valid(L, t)) v = prm.p[wp][(int64_t)row * weight_K(wp) + col];
    } else {
      // A[i = forward in-feature (r)][p = forward out-feature of forward tile t (ar)]
      const int s = bwd_unit_stage(u), j = u - bwd_unit_first(s), L = bwd_fwd_layer(s);
      const int wp = fwd_out_weight(L, t);
      const int row = fwd_out_row0(L, t) + ar, col = bwd_out_colbase(s, j) + r;
      if (ar < fwd_out_valid(L, t)) v = prm.p[wp][(int64_t)row * weight_K(wp) + col];
    }
    vals[e] = P::cvt(v);
  }
#pragma unroll
  for (int e = 0; e < P::E; ++e) ((typename P::Store*)dst)[e] = vals[e];
}

// ------------------------------------------------------------------------------------
// weight stream: 2-slot LDS ring filled by global_load_lds (1 KiB per wave-instruction)
// ------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gsrc, (lds_void*)lds_wave_base, 16, 0, 0);
}

// The same LDS-DMA hidden from hipcc's waitcnt bookkeeping: hipcc waits vmcnt(0) before
// any ds_read_tr while one of its own LDS-DMAs is pending, which would drain a multi-block
// ring.  The caller owns completion (counted s_waitcnt vmcnt + s_barrier before reading).
__device__ __forceinline__ void glds16_asm(const void* gsrc, uint32_t lds_wave_base) {
  uint32_t saved;  // m0 is reserved to the compiler: save and restore it around the DMA
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_wave_base)) : "memory");
}

template <class P, int SLOT_CHUNKS>
struct Stream {
  const uint4* g;  // chunk c of the packed buffer starts at g + 64 c
  uint4* lds;
  int slot;
  // issue the copy of `n` chunks starting at global chunk `c0` into slot `to`
  __device__ __forceinline__ void fetch(int c0, int n, int to) const {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int k = wave; k < n; k += P::WAVES)
      glds16(g + (int64_t)(c0 + k) * 64 + lane, lds + (to * SLOT_CHUNKS + k) * 64);
  }
  __device__ __forceinline__ const uint4* cur() const { return lds + slot * SLOT_CHUNKS * 64; }
};

template <class P>
__device__ __forceinline__ f32x16 tile_mma(const uint4* slot_base, int tile_idx, const typename P::Tile& b,
                                           f32x16 acc, int lane) {
#pragma unroll
  for (int c = 0; c < P::CH; ++c) {
    uint4 a = slot_base[(tile_idx * P::CH + c) * 64 + lane];
    acc = P::mma(a, b, c, acc);
  }
  return acc;
}

// ------------------------------------------------------------------------------------
// positional encoding straight into accumulator-layout tiles
// (freq.py:7-32: [x, sin(2^k x), cos(2^k x)]_k; feature 3 + 6k + {0..2 sin, 3..5 cos})
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float pe_feature(int f, int nfreq, float x0, float x1, float x2) {
  if (f < 3) return f == 0 ? x0 : f == 1 ? x1 : x2;
  const int g = f - 3;
  const int k = g / 6, r = g - 6 * k;
  if (k >= nfreq) return 0.f;
  const int dim = r % 3;
  const float x = dim == 0 ? x0 : dim == 1 ? x1 : x2;
  const float a = x * (float)(1 << k);  // exact power-of-two scale, as x * 2.**k in torch
  return r < 3 ? sinf(a) : cosf(a);
}

template <class P>
__device__ __forceinline__ void pe_tile(typename P::Tile& t, int tile, int nfreq, int nvalid, int h, float x0,
                                        float x1, float x2) {
#pragma unroll
  for (int rho = 0; rho < 16; ++rho) {
    const int f = 32 * tile + acc_row(rho, h);
    P::set(t, rho, f < nvalid ? pe_feature(f, nfreq, x0, x1, x2) : 0.f);
  }
}

// fragment-native store of one finished tile (mlp_tables.h, "Training stores"): CH
// lane-linear 16-byte stores per lane, each wave-instruction writes 1 KiB contiguous
template <class P>
__device__ __forceinline__ void store_tile(void* base, int64_t nblk, int tau, int64_t wblock, int lane,
                                           const typename P::Tile& t) {
  uint4* dst = (uint4*)base + ((int64_t)tau * nblk + wblock) * P::CH * 64 + lane;
#pragma unroll
  for (int c = 0; c < P::CH; ++c) dst[c * 64] = P::chunk(t, c);
}

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
  uint16_t* masks;           // [nblk, MASK_TILES, 64] or null
};

// activation of a finished accumulator tile -> next layer's B operand (+ training stores)
template <class P, bool RELU, bool STORE>
__device__ __forceinline__ void finish_tile(const f32x16& acc, typename P::Tile& out, const FwdArgs& a, int act_tile,
                                            int mask_tile, int64_t m, int64_t wblock, int h, int lane) {
  uint32_t mask = 0;
#pragma unroll
  for (int rho = 0; rho < 16; ++rho) {
    float x = acc[rho];
    if (RELU) {
      mask |= (x > 0.f ? 1u : 0u) << rho;
      x = x > 0.f ? x : 0.f;
    }
    P::set(out, rho, x);
  }
  if (STORE) {
    store_tile<P>(a.act, a.nblk, act_tile, wblock, lane, out);
    if (RELU) a.masks[(wblock * MASK_TILES + mask_tile) * 64 + lane] = (uint16_t)mask;
  }
}

__device__ __forceinline__ f32x16 bias_init(const uint4* bias_chunk, int h) {
  f32x16 acc;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // rows 8q + 4h + {0..3} = floats [8q+4h, 8q+4h+4) = lane (2q + h) of the bias chunk
    uint4 b = bias_chunk[2 * q + h];
    acc[4 * q + 0] = __uint_as_float(b.x);
    acc[4 * q + 1] = __uint_as_float(b.y);
    acc[4 * q + 2] = __uint_as_float(b.z);
    acc[4 * q + 3] = __uint_as_float(b.w);
  }
  return acc;
}

template <class P> __host__ __device__ constexpr int fwd_slot_chunks() { return 10 * P::CH + 1; }
template <class P> __host__ __device__ constexpr int dx_slot_chunks() { return 9 * P::CH; }

// Forward.  Unit sequence = fwd_unit_*; the density-only variant (grid bake: only
// raw[...,3] is used, occupancy_grid.py:60) jumps from the last trunk unit to alpha.
template <class P, bool STORE, bool DENSITY>
__global__ void __launch_bounds__(P::WAVES * 64) fwd_kernel(FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem_u4[];
  using Tile = typename P::Tile;
  constexpr int SC = fwd_slot_chunks<P>();
  Stream<P, SC> ws{(const uint4*)a.wpack, smem_u4, 0};

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int64_t wblock = (int64_t)blockIdx.x * P::WAVES + wave;
  const int64_t m = wblock * 32 + c;
  const int64_t ms = m < a.M ? m : a.M - 1;

  constexpr int U_ALPHA = fwd_unit_first(LFA) + 8;
  auto next_unit = [](int u) -> int {
    if (DENSITY) {
      if (u == fwd_unit_first(LFA) - 1) return U_ALPHA;
      if (u == U_ALPHA) return -1;
    }
    return u + 1 < NUNIT_FWD ? u + 1 : -1;
  };
  f32x16 acc;
  auto begin = [&](int u) {
    const int nu = next_unit(u);
    if (nu >= 0) ws.fetch(fwd_unit_chunk_off(nu, P::CH), fwd_unit_chunks(nu, P::CH), ws.slot ^ 1);
    acc = bias_init(ws.cur() + fwd_unit_tiles(u) * P::CH * 64, h);
  };
  auto end = [&]() {
    __syncthreads();  // vmcnt(0): next unit landed; everyone is done reading this slot
    ws.slot ^= 1;
  };

  ws.fetch(fwd_unit_chunk_off(0, P::CH), fwd_unit_chunks(0, P::CH), 0);

  const float px = a.pts[ms * 3 + 0], py = a.pts[ms * 3 + 1], pz = a.pts[ms * 3 + 2];
  float dx = 0.f, dy = 0.f, dz = 0.f;
  if (!DENSITY) {
    const int64_t di = a.dir_index ? (int64_t)a.dir_index[ms] : ms / a.samples_per_dir;
    dx = a.dirs[di * 3 + 0];
    dy = a.dirs[di * 3 + 1];
    dz = a.dirs[di * 3 + 2];
  }
  Tile Ha[8], Hb[8];
  {
    Tile X[2];
    pe_tile<P>(X[0], 0, 10, 63, h, px, py, pz);
    pe_tile<P>(X[1], 1, 10, 63, h, px, py, pz);
    if (STORE) {
      Tile D;
      pe_tile<P>(D, 0, 4, 27, h, dx, dy, dz);
      store_tile<P>(a.act, a.nblk, AT_X, wblock, lane, X[0]);
      store_tile<P>(a.act, a.nblk, AT_X + 1, wblock, lane, X[1]);
      store_tile<P>(a.act, a.nblk, AT_D, wblock, lane, D);
    }
    __syncthreads();
    int unit = 0;
    // ---- L0: PE(xyz) -> Ha
#pragma unroll
    for (int n = 0; n < 8; ++n, ++unit) {
      begin(unit);
      acc = tile_mma<P>(ws.cur(), 0, X[0], acc, lane);
      acc = tile_mma<P>(ws.cur(), 1, X[1], acc, lane);
      end();
      finish_tile<P, true, STORE>(acc, Ha[n], a, AT_H + n, n, m, wblock, h, lane);
    }
  }
  int unit = 8;
  // ---- L1..L4 (ping-pong: L1 Ha->Hb, L2 Hb->Ha, L3 Ha->Hb, L4 Hb->Ha)
#define NERF_HIDDEN_LAYER(L, IN, OUT)                                                            \
  _Pragma("unroll") for (int n = 0; n < 8; ++n, ++unit) {                                        \
    begin(unit);                                                                                 \
    _Pragma("unroll") for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), t, IN[t], acc, lane); \
    end();                                                                                       \
    finish_tile<P, true, STORE>(acc, OUT[n], a, AT_H + (L) * 8 + n, (L) * 8 + n, m, wblock, h, lane);     \
  }
  NERF_HIDDEN_LAYER(1, Ha, Hb)
  NERF_HIDDEN_LAYER(2, Hb, Ha)
  NERF_HIDDEN_LAYER(3, Ha, Hb)
  NERF_HIDDEN_LAYER(4, Hb, Ha)
  // ---- L5: [PE(xyz), h4] -> Hb   (PE recomputed instead of held through L1..L4)
  {
    Tile X[2];
    pe_tile<P>(X[0], 0, 10, 63, h, px, py, pz);
    pe_tile<P>(X[1], 1, 10, 63, h, px, py, pz);
#pragma unroll
    for (int n = 0; n < 8; ++n, ++unit) {
      begin(unit);
      acc = tile_mma<P>(ws.cur(), 0, X[0], acc, lane);
      acc = tile_mma<P>(ws.cur(), 1, X[1], acc, lane);
#pragma unroll
      for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), 2 + t, Ha[t], acc, lane);
      end();
      finish_tile<P, true, STORE>(acc, Hb[n], a, AT_H + 5 * 8 + n, 5 * 8 + n, m, wblock, h, lane);
    }
  }
  NERF_HIDDEN_LAYER(6, Hb, Ha)
  NERF_HIDDEN_LAYER(7, Ha, Hb)
#undef NERF_HIDDEN_LAYER
  // ---- feature (no activation) -> Ha ; alpha (output row 0: lanes 0..31, register 0)
  if (!DENSITY) {
#pragma unroll
    for (int n = 0; n < 8; ++n, ++unit) {
      begin(unit);
#pragma unroll
      for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), t, Hb[t], acc, lane);
      end();
      finish_tile<P, false, STORE>(acc, Ha[n], a, AT_F + n, 0, m, wblock, h, lane);
    }
  } else {
    unit += 8;
  }
  float alpha;
  {
    begin(unit);
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), t, Hb[t], acc, lane);
    end();
    alpha = acc[0];
    ++unit;
  }
  if (DENSITY) {
    if (h == 0 && m < a.M) *(float4*)(a.raw + m * 4) = make_float4(0.f, 0.f, 0.f, alpha);
    return;
  }
  // ---- views: [feature, PE(dir)] -> Hb[0..3]
  {
    Tile D;
    pe_tile<P>(D, 0, 4, 27, h, dx, dy, dz);
#pragma unroll
    for (int n = 0; n < 4; ++n, ++unit) {
      begin(unit);
#pragma unroll
      for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), t, Ha[t], acc, lane);
      acc = tile_mma<P>(ws.cur(), 8, D, acc, lane);
      end();
      finish_tile<P, true, STORE>(acc, Hb[n], a, AT_V + n, 64 + n, m, wblock, h, lane);
    }
  }
  // ---- rgb (rows 0..2: lanes 0..31, registers 0..2)
  begin(unit);
#pragma unroll
  for (int t = 0; t < 4; ++t) acc = tile_mma<P>(ws.cur(), t, Hb[t], acc, lane);
  end();
  if (h == 0 && m < a.M) *(float4*)(a.raw + m * 4) = make_float4(acc[0], acc[1], acc[2], alpha);
}

// ------------------------------------------------------------------------------------
// backward dX chain
// ------------------------------------------------------------------------------------
struct DxArgs {
  const char* wpack_t;  // W^T chunks
  const float* d_raw;   // [M,4]
  int64_t M, nblk;
  const uint16_t* masks;
  void* dz;             // [ZT_TILES][nblk] tile-blocks
};

template <class P, bool MASK>
__device__ __forceinline__ void dx_finish(const f32x16& acc, typename P::Tile& out, const DxArgs& a, int dz_tile,
                                          int mask_tile, int64_t m, int64_t wblock, int h, int lane) {
  const uint32_t mask = MASK ? (uint32_t)a.masks[(wblock * MASK_TILES + mask_tile) * 64 + lane] : 0xFFFFu;
#pragma unroll
  for (int rho = 0; rho < 16; ++rho) P::set(out, rho, ((mask >> rho) & 1u) ? acc[rho] : 0.f);
  store_tile<P>(a.dz, a.nblk, dz_tile, wblock, lane, out);
}

template <class P>
__global__ void __launch_bounds__(P::WAVES * 64) dx_kernel(DxArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem_u4[];
  using Tile = typename P::Tile;
  constexpr int SC = dx_slot_chunks<P>();
  Stream<P, SC> ws{(const uint4*)a.wpack_t, smem_u4, 0};
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int64_t wblock = (int64_t)blockIdx.x * P::WAVES + wave;
  const int64_t m = wblock * 32 + c;

  f32x16 acc;
  auto begin = [&](int u) {
    if (u + 1 < NUNIT_BWD) ws.fetch(bwd_unit_chunk_off(u + 1, P::CH), bwd_unit_chunks(u + 1, P::CH), ws.slot ^ 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  };
  auto end = [&]() {
    __syncthreads();
    ws.slot ^= 1;
  };

  ws.fetch(bwd_unit_chunk_off(0, P::CH), bwd_unit_chunks(0, P::CH), 0);

  // output gradients of rgb_linear (rows 0..2) and alpha_linear (row 0): lanes 0..31
  const float4 g = m < a.M ? *(const float4*)(a.d_raw + m * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  Tile G, DA;
#pragma unroll
  for (int rho = 0; rho < 16; ++rho) {
    P::set(G, rho, (h == 0 && rho < 3) ? (rho == 0 ? g.x : rho == 1 ? g.y : g.z) : 0.f);
    P::set(DA, rho, (h == 0 && rho == 0) ? g.w : 0.f);
  }
  store_tile<P>(a.dz, a.nblk, ZT_RGB, wblock, lane, G);
  store_tile<P>(a.dz, a.nblk, ZT_A, wblock, lane, DA);
  __syncthreads();

  Tile Ha[8], Hb[8];
  int unit = 0;
  // bRGB: dhv = W_rgb^T drgb, masked by hv > 0 -> dZv (Hb[0..3])
#pragma unroll
  for (int j = 0; j < 4; ++j, ++unit) {
    begin(unit);
    acc = tile_mma<P>(ws.cur(), 0, G, acc, lane);
    end();
    dx_finish<P, true>(acc, Hb[j], a, ZT_V + j, 64 + j, m, wblock, h, lane);
  }
  // bV: dfeature = W_v[:, :256]^T dZv -> Ha
#pragma unroll
  for (int j = 0; j < 8; ++j, ++unit) {
    begin(unit);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc = tile_mma<P>(ws.cur(), t, Hb[t], acc, lane);
    end();
    dx_finish<P, false>(acc, Ha[j], a, ZT_F + j, 0, m, wblock, h, lane);
  }
  // bFA: dh7 = W_f^T dfeature + W_a^T dalpha, masked by h7 -> dZ7 (Hb)
#pragma unroll
  for (int j = 0; j < 8; ++j, ++unit) {
    begin(unit);
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), t, Ha[t], acc, lane);
    acc = tile_mma<P>(ws.cur(), 8, DA, acc, lane);
    end();
    dx_finish<P, true>(acc, Hb[j], a, ZT_H + 7 * 8 + j, 7 * 8 + j, m, wblock, h, lane);
  }
  // b_l (l = 7..1): dh_{l-1} = W_l^T dZ_l (L5: h4 columns only), masked by h_{l-1}
#define NERF_BWD_LAYER(L, IN, OUT)                                                                \
  _Pragma("unroll") for (int j = 0; j < 8; ++j, ++unit) {                                         \
    begin(unit);                                                                                  \
    _Pragma("unroll") for (int t = 0; t < 8; ++t) acc = tile_mma<P>(ws.cur(), t, IN[t], acc, lane); \
    end();                                                                                        \
    dx_finish<P, true>(acc, OUT[j], a, ZT_H + ((L) - 1) * 8 + j, ((L) - 1) * 8 + j, m, wblock, h, lane);       \
  }
  NERF_BWD_LAYER(7, Hb, Ha)
  NERF_BWD_LAYER(6, Ha, Hb)
  NERF_BWD_LAYER(5, Hb, Ha)
  NERF_BWD_LAYER(4, Ha, Hb)
  NERF_BWD_LAYER(3, Hb, Ha)
  NERF_BWD_LAYER(2, Ha, Hb)
  NERF_BWD_LAYER(1, Hb, Ha)
#undef NERF_BWD_LAYER
}

// ------------------------------------------------------------------------------------
// dW / db: C[n][k] += sum_m dz[n][m] act[k][m] over a chunk of 32-sample blocks.
// job = (gemm g, n-group, k-group, block chunk); wave w owns n-tile w of the group and
// accumulates all (<= 8) k-tiles of the group.  Per block, the group's dz and act
// tile-blocks (fragment-native, mlp_tables.h) are copied to LDS with global_load_lds and
// read back transposed: K = samples.  Row i of a fragment <-> feature acc_row(i&15, i>>4).
// ------------------------------------------------------------------------------------
struct DwArgs {
  const void* dz;
  const void* act;
  int64_t nblk;       // 32-sample blocks in the stores
  int64_t chunk_blk;  // blocks per job
  int nchunks;
  float* grad;        // flat [NET_PARAMS], accumulated
};

struct DwJob { int g, ng, kg; };

__host__ __device__ constexpr int gemm_ngroups(int g) { return (gemm_n_tiles(g) + 7) / 8; }
__host__ __device__ constexpr int gemm_kgroups(int g) { return (gemm_k_tiles(g) + 7) / 8; }
__host__ __device__ constexpr int n_dw_jobs_per_chunk() {
  int n = 0;
  for (int g = 0; g < NGEMM; ++g) n += gemm_ngroups(g) * gemm_kgroups(g);
  return n;
}
__device__ __forceinline__ DwJob dw_job(int j) {
  for (int g = 0; g < NGEMM; ++g) {
    const int n = gemm_ngroups(g) * gemm_kgroups(g);
    if (j < n) return DwJob{g, j / gemm_kgroups(g), j % gemm_kgroups(g)};
    j -= n;
  }
  return DwJob{0, 0, 0};
}

constexpr int DW_WAVES = 8;
constexpr int DW_SLOTS = 16;  // 8 dz tiles + 8 act tiles per block
__host__ __device__ constexpr int perm_row(int i) { return acc_row(i & 15, i >> 4); }
// LDS ring depth: 3 x 32 KiB (bf16), 2 x 64 KiB (fp32) -- both within 160 KiB
template <class P> __host__ __device__ constexpr int dw_nbuf() { return P::CH == 2 ? 3 : 2; }

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 8]
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((address_space(3))) short4_t lds_short4;

// bf16: the 8-sample K fragment (samples 16 s + 8 h + [0, 8)) of row (lane & 31)
__device__ __forceinline__ bf16x8 dw_frag_bf16(const char* tile, int s, int lane) {
  const int l16 = lane & 15, G = lane >> 4;
  const int hp = G & 1, h = G >> 1, q = l16 >> 2, pp = l16 & 3;
  const char* base = tile + (pp >> 1) * 1024 + (pp & 1) * 8 + (16 * s + 8 * h + q + 32 * hp) * 16;
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)base);
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(base + 4 * 16));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
// fp32: the K = 2 fragment (sample 2 s + h) of row (lane & 31)
__device__ __forceinline__ float dw_frag_f32(const char* tile, int s, int lane) {
  const int rho = lane & 15, hp = (lane >> 4) & 1, h = lane >> 5;
  return *(const float*)(tile + (rho >> 2) * 1024 + (2 * s + h + 32 * hp) * 16 + (rho & 3) * 4);
}

template <class P>
__global__ void __launch_bounds__(DW_WAVES * 64) dw_kernel(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 smem_u4[];
  constexpr int TB = P::CH * 1024;           // tile-block bytes
  constexpr int BUF = DW_SLOTS * TB;         // one block's tiles
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int chunk_id = blockIdx.x % a.nchunks;
  const DwJob job = dw_job(blockIdx.x / a.nchunks);
  const int g = job.g;
  const int nt0 = job.ng * 8, kt0 = job.kg * 8;
  const int ntiles = min(8, gemm_n_tiles(g) - nt0);
  const int ktiles = min(8, gemm_k_tiles(g) - kt0);
  const bool active = wave < ntiles;
  const int64_t b_begin = (int64_t)chunk_id * a.chunk_blk;
  const int64_t b_end = min(b_begin + a.chunk_blk, a.nblk);
  char* lds = (char*)smem_u4;

  // copy one block's tile-blocks into buffer `buf` (each wave-instruction = 1 KiB).  Wave w
  // issues chunks k = w, w + 8, ... (G of them); their sources and LDS offsets are resolved
  // once here -- a table lookup inside the loop would be an ordinary global load, whose
  // compiler wait is vmcnt(0) and drains the ring.
  const int nchunk = (ntiles + ktiles) * P::CH;
  constexpr int GMAX = 16 * P::CH / DW_WAVES;
  const int G = wave < nchunk ? (nchunk - wave + DW_WAVES - 1) / DW_WAVES : 0;
  const char* src[GMAX];
  int dst[GMAX];
#pragma unroll
  for (int i = 0; i < GMAX; ++i) {
    const int k = wave + DW_WAVES * i;
    const int which = k / P::CH, c = k % P::CH;
    const bool is_a = which < ntiles;
    const int slot = is_a ? which : 8 + (which - ntiles);
    const int tau = k >= nchunk ? 0 : is_a ? gemm_dz_tile(g, nt0 + which) : gemm_act_tile(g, kt0 + which - ntiles);
    src[i] = (const char*)(is_a ? a.dz : a.act) + ((int64_t)tau * a.nblk * P::CH + c) * 1024 + lane * 16;
    dst[i] = slot * TB + c * 1024;
  }
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_void*)lds;
  auto fetch = [&](int64_t b, int buf) {
    const int64_t boff = b * (P::CH * 1024);
#pragma unroll
    for (int i = 0; i < GMAX; ++i)
      if (i < G) glds16_asm(src[i] + boff, lds_base + buf * BUF + dst[i]);
  };

  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
  float dbias = 0.f;

  // NBUF-slot ring, D = NBUF - 1 blocks in flight: per block each wave issues the same
  // number G of global_load_lds, so "block b landed" = vmcnt(G * younger blocks in flight),
  // then a raw s_barrier -- no vmcnt(0) drain (cdna_hip_programming.md, LDS-DMA ordering).
  constexpr int NBUF = dw_nbuf<P>(), D = NBUF - 1;
  for (int d = 0; d < D; ++d)
    if (b_begin + d < b_end) fetch(b_begin + d, d);
  int buf = 0;
  for (int64_t b = b_begin; b < b_end; ++b) {
    const int younger = (int)min((int64_t)(D - 1), b_end - 1 - b);
    wait_vmcnt(G * younger);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (b + D < b_end) fetch(b + D, buf == 0 ? NBUF - 1 : buf - 1);
    if (active) {
      const char* tiles = lds + buf * BUF;
      const char* at = tiles + wave * TB;
      if constexpr (P::CH == 2) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 af = dw_frag_bf16(at, s, lane);
#pragma unroll
          for (int e = 0; e < 8; ++e) dbias += (float)af[e];
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (t < ktiles)
              acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, dw_frag_bf16(tiles + (8 + t) * TB, s, lane), acc[t],
                                                               0, 0, 0);
        }
      } else {
#pragma unroll 4
        for (int s = 0; s < 16; ++s) {
          const float af = dw_frag_f32(at, s, lane);
          dbias += af;
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (t < ktiles)
              acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, dw_frag_f32(tiles + (8 + t) * TB, s, lane), acc[t], 0,
                                                            0, 0);
        }
      }
    }
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }
  if (!active) return;
  // accumulate into the flat gradient (state_dict layout: weight [N][K] row-major)
  const int wp = gemm_weight(g);
  float* gw = a.grad + param_offset(wp);
  const int K = weight_K(wp);
  const int nvalid = gemm_n_valid(g);
  const int h = lane >> 5, j = lane & 31;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    if (t < ktiles) {
      const int kt = kt0 + t;
      const int colf = perm_row(j);
      const int col = gemm_col0(g, kt) + colf;
      const bool cok = colf < gemm_col_valid(g, kt);
#pragma unroll
      for (int rho = 0; rho < 16; ++rho) {
        const int n = 32 * (nt0 + wave) + perm_row(acc_row(rho, h));
        if (cok && n < nvalid) atomicAdd(gw + (int64_t)n * K + col, acc[t][rho]);
      }
    }
  }
  if (job.kg == 0) {
    dbias += __shfl_xor(dbias, 32, 64);
    const int n = 32 * (nt0 + wave) + perm_row(j);
    if (h == 0 && n < nvalid) atomicAdd(a.grad + param_offset(wp + 1) + n, dbias);
  }
}

}  // namespace mlp
}  // namespace nerf

// ======================================================================================
// C-ABI
// ======================================================================================
using namespace nerf;
using namespace nerf::mlp;

template <class P> static constexpr size_t fwd_lds_bytes() { return 2 * (size_t)fwd_slot_chunks<P>() * 1024; }
template <class P> static constexpr size_t dx_lds_bytes() { return 2 * (size_t)dx_slot_chunks<P>() * 1024; }
template <class P> static constexpr size_t dw_lds_bytes() { return (size_t)dw_nbuf<P>() * DW_SLOTS * P::CH * 1024; }

template <class K>
static void allow_lds(K kernel, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

extern "C" {

int64_t nerf_mlp_net_params(void) { return NET_PARAMS; }
int64_t nerf_mlp_param_offset(int i) { return (i >= 0 && i <= NPARAM) ? param_offset(i) : -1; }

int64_t nerf_mlp_packed_bytes(int dtype, int dir) {
  if ((dtype != 0 && dtype != 1) || (dir != 0 && dir != 1)) return -1;
  return total_chunks(dtype == 0 ? PF32::CH : PBF16::CH, dir) * 1024;
}

int64_t nerf_mlp_padded_samples(int64_t M) { return (M + M_ALIGN - 1) / M_ALIGN * M_ALIGN; }
int64_t nerf_mlp_act_bytes(int dtype, int64_t M) {
  return (int64_t)A_ROWS * nerf_mlp_padded_samples(M) * (dtype == 0 ? 4 : 2);
}
int64_t nerf_mlp_dz_bytes(int dtype, int64_t M) {
  return (int64_t)Z_ROWS * nerf_mlp_padded_samples(M) * (dtype == 0 ? 4 : 2);
}
int64_t nerf_mlp_mask_bytes(int64_t M) { return nerf_mlp_padded_samples(M) / 32 * MASK_TILES * 64 * 2; }

int nerf_mlp_pack(const float* const* params, int dtype, void* packed_fwd, void* packed_bwd, hipStream_t stream) {
  NERF_REQUIRE(params != nullptr, "nerf_mlp_pack: params is null");
  NERF_REQUIRE(dtype == 0 || dtype == 1, "nerf_mlp_pack: dtype must be 0 (f32) or 1 (bf16), got %d", dtype);
  ParamPtrs prm;
  for (int i = 0; i < NPARAM; ++i) {
    NERF_REQUIRE(params[i] != nullptr, "nerf_mlp_pack: params[%d] is null", i);
    prm.p[i] = params[i];
  }
  const int ch = dtype == 0 ? PF32::CH : PBF16::CH;
  for (int dir = 0; dir < 2; ++dir) {
    void* dst = dir == 0 ? packed_fwd : packed_bwd;
    if (!dst) continue;
    const int64_t n = total_chunks(ch, dir) * 64;
    dim3 grid((unsigned)((n + 255) / 256));
    if (dtype == 0) {
      if (dir == 0) hipLaunchKernelGGL((pack_kernel<PF32, 0>), grid, dim3(256), 0, stream, prm, (char*)dst);
      else hipLaunchKernelGGL((pack_kernel<PF32, 1>), grid, dim3(256), 0, stream, prm, (char*)dst);
    } else {
      if (dir == 0) hipLaunchKernelGGL((pack_kernel<PBF16, 0>), grid, dim3(256), 0, stream, prm, (char*)dst);
      else hipLaunchKernelGGL((pack_kernel<PBF16, 1>), grid, dim3(256), 0, stream, prm, (char*)dst);
    }
    if (int e = check_launch("nerf_mlp_pack")) return e;
  }
  return 0;
}

// flags: bit0 = store activations + masks for backward, bit1 = density only
int nerf_mlp_fwd(const void* packed_fwd, int dtype, const float* pts, const float* viewdirs, int samples_per_dir,
                 const int32_t* dir_index, int64_t M, int flags, float* raw, void* act, uint16_t* masks,
                 hipStream_t stream) {
  NERF_REQUIRE(dtype == 0 || dtype == 1, "nerf_mlp_fwd: bad dtype %d", dtype);
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
  if (dtype == 0) {
    using P = PF32;
    const int spb = samples_per_block<P>();
    dim3 grid((unsigned)(store ? a.nblk * 32 / spb : (M + spb - 1) / spb));
    const size_t lds = fwd_lds_bytes<P>();
    if (store) {
      allow_lds(fwd_kernel<P, true, false>, lds);
      hipLaunchKernelGGL((fwd_kernel<P, true, false>), grid, dim3(P::WAVES * 64), lds, stream, a);
    } else if (density) {
      allow_lds(fwd_kernel<P, false, true>, lds);
      hipLaunchKernelGGL((fwd_kernel<P, false, true>), grid, dim3(P::WAVES * 64), lds, stream, a);
    } else {
      allow_lds(fwd_kernel<P, false, false>, lds);
      hipLaunchKernelGGL((fwd_kernel<P, false, false>), grid, dim3(P::WAVES * 64), lds, stream, a);
    }
  } else {
    using P = PBF16;
    const int spb = samples_per_block<P>();
    dim3 grid((unsigned)(store ? a.nblk * 32 / spb : (M + spb - 1) / spb));
    const size_t lds = fwd_lds_bytes<P>();
    if (store) hipLaunchKernelGGL((fwd_kernel<P, true, false>), grid, dim3(P::WAVES * 64), lds, stream, a);
    else if (density) hipLaunchKernelGGL((fwd_kernel<P, false, true>), grid, dim3(P::WAVES * 64), lds, stream, a);
    else hipLaunchKernelGGL((fwd_kernel<P, false, false>), grid, dim3(P::WAVES * 64), lds, stream, a);
  }
  return check_launch("nerf_mlp_fwd");
}

int64_t nerf_mlp_dw_chunk(int64_t M) {
  // samples per dW job (multiple of 256): >= 8 chunks so every CU gets work, <= 16384
  const int64_t ldm = nerf_mlp_padded_samples(M);
  int64_t ch = 16384;
  while (ch > 256 && ldm / ch < 8) ch /= 2;
  return ch;
}

// dX chain only: dz (per-layer output gradients, fragment-native tiles) from d_raw + masks
int nerf_mlp_bwd_dx(const void* packed_bwd, int dtype, const float* d_raw, int64_t M, const uint16_t* masks, void* dz,
                    hipStream_t stream) {
  NERF_REQUIRE(dtype == 0 || dtype == 1, "nerf_mlp_bwd_dx: bad dtype %d", dtype);
  NERF_REQUIRE(M >= 0, "nerf_mlp_bwd_dx: M < 0");
  if (M == 0) return 0;
  NERF_REQUIRE(packed_bwd && d_raw && masks && dz, "nerf_mlp_bwd_dx: null pointer");
  const int64_t ldm = nerf_mlp_padded_samples(M);
  DxArgs x{(const char*)packed_bwd, d_raw, M, ldm / 32, masks, dz};
  if (dtype == 0) {
    using P = PF32;
    allow_lds(dx_kernel<P>, dx_lds_bytes<P>());
    hipLaunchKernelGGL((dx_kernel<P>), dim3((unsigned)(ldm / samples_per_block<P>())), dim3(P::WAVES * 64),
                       dx_lds_bytes<P>(), stream, x);
  } else {
    using P = PBF16;
    hipLaunchKernelGGL((dx_kernel<P>), dim3((unsigned)(ldm / samples_per_block<P>())), dim3(P::WAVES * 64),
                       dx_lds_bytes<P>(), stream, x);
  }
  return check_launch("nerf_mlp_bwd_dx");
}

// dW/db only: grad += dz . act^T (grad must be zeroed or hold a running sum)
int nerf_mlp_bwd_dw(int dtype, int64_t M, const void* act, const void* dz, float* grad, hipStream_t stream) {
  NERF_REQUIRE(dtype == 0 || dtype == 1, "nerf_mlp_bwd_dw: bad dtype %d", dtype);
  NERF_REQUIRE(M >= 0, "nerf_mlp_bwd_dw: M < 0");
  if (M == 0) return 0;
  NERF_REQUIRE(act && dz && grad, "nerf_mlp_bwd_dw: null pointer");
  const int64_t nblk = nerf_mlp_padded_samples(M) / 32;
  const int64_t chunk_blk = nerf_mlp_dw_chunk(M) / 32;
  const int nchunks = (int)((nblk + chunk_blk - 1) / chunk_blk);
  DwArgs w{dz, act, nblk, chunk_blk, nchunks, grad};
  dim3 grid((unsigned)(n_dw_jobs_per_chunk() * nchunks));
  if (dtype == 0) {
    allow_lds(dw_kernel<PF32>, dw_lds_bytes<PF32>());
    hipLaunchKernelGGL((dw_kernel<PF32>), grid, dim3(DW_WAVES * 64), dw_lds_bytes<PF32>(), stream, w);
  } else {
    allow_lds(dw_kernel<PBF16>, dw_lds_bytes<PBF16>());
    hipLaunchKernelGGL((dw_kernel<PBF16>), grid, dim3(DW_WAVES * 64), dw_lds_bytes<PBF16>(), stream, w);
  }
  return check_launch("nerf_mlp_bwd_dw");
}

int nerf_mlp_bwd(const void* packed_bwd, int dtype, const float* d_raw, int64_t M, const void* act,
                 const uint16_t* masks, void* dz, float* grad, hipStream_t stream) {
  if (int e = nerf_mlp_bwd_dx(packed_bwd, dtype, d_raw, M, masks, dz, stream)) return e;
  return nerf_mlp_bwd_dw(dtype, M, act, dz, grad, stream);
}

}  // extern "C"
