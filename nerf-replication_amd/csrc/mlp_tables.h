// Compile-time layout of the lego NeRF MLP on MFMA tiles.
//
// Reference: src/models/nerf/network.py:9-74 (NeRF: D=8, W=256, skips=[4], use_viewdirs)
// with the frequency encoders of src/models/encoding/freq.py (xyz L=10 -> 63, dir L=4 -> 27).
//
// Every matrix product is computed "feature-major": an accumulator tile is 32 features x
// 32 samples (v_mfma_f32_32x32x{16_bf16,2_f32}); lane l holds sample (l & 31) and, in
// its 16 accumulator registers rho, feature acc_row(rho, l >> 5).  A layer's input is a
// list of such 32-feature tiles (the previous layer's accumulators, or the positional
// encoding laid out the same way), so one layer's output feeds the next MFMA's B
// operand straight from registers.  Weights (A operand) are re-packed once per optimizer
// step into 1 KiB lane-linear "chunks" (64 lanes x 16 B) in exactly that k order.
#pragma once
#include <stdint.h>

namespace nerf {
namespace mlp {

__host__ __device__ constexpr int acc_row(int rho, int h) { return (rho & 3) + 8 * (rho >> 2) + 4 * h; }

// forward layers (in execution order)
enum Layer { L0 = 0, L1, L2, L3, L4, L5, L6, L7, LFA, LV, LRGB, NLAYER };

// parameter slots, state_dict order of one NeRF (network.py:22-44)
enum Param {
  P_W0 = 0,  // pts_linears.i.weight = 2i, .bias = 2i+1 (i = 0..7)
  P_VW = 16, P_VB = 17,   // views_linears.0
  P_FW = 18, P_FB = 19,   // feature_linear
  P_AW = 20, P_AB = 21,   // alpha_linear
  P_RW = 22, P_RB = 23,   // rgb_linear
  NPARAM = 24
};

// in_features of each weight (row stride of nn.Linear's [out, in] weight)
__host__ __device__ constexpr int weight_K(int p) {
  return p == 0 ? 63 : p == 10 ? 319 : p == P_VW ? 283 : p == P_RW ? 128 : 256;
}
__host__ __device__ constexpr int weight_N(int p) {
  return p == P_VW ? 128 : p == P_AW ? 1 : p == P_RW ? 3 : 256;
}
// element offsets of every parameter in the flat state_dict-order gradient buffer
__host__ __device__ constexpr int64_t param_numel(int i) {
  return (i & 1) ? weight_N(i - 1) : (int64_t)weight_N(i) * weight_K(i);
}
__host__ __device__ constexpr int64_t param_offset(int i) {
  int64_t o = 0;
  for (int k = 0; k < i; ++k) o += param_numel(k);
  return o;
}
constexpr int64_t NET_PARAMS = param_offset(NPARAM);  // 595,844
static_assert(NET_PARAMS == 595844, "NeRF parameter count");

// number of input tiles / output tiles per forward layer
__host__ __device__ constexpr int fwd_in_tiles(int L) {
  return L == L0 ? 2 : L == L5 ? 10 : L == LV ? 9 : L == LRGB ? 4 : 8;
}
__host__ __device__ constexpr int fwd_out_tiles(int L) {
  return L == LFA ? 9 : L == LV ? 4 : L == LRGB ? 1 : 8;
}
// input tile t of layer L -> (first weight column, number of valid columns)
__host__ __device__ constexpr int fwd_in_colbase(int L, int t) {
  return L == L0 ? 32 * t
       : L == L5 ? (t < 2 ? 32 * t : 63 + 32 * (t - 2))
       : L == LV ? 32 * t
       : 32 * t;
}
__host__ __device__ constexpr int fwd_in_valid(int L, int t) {
  return (L == L0 || L == L5) && t == 1 ? 31 : (L == LV && t == 8) ? 27 : 32;
}
// output tile n of layer L -> weight param, first weight row, valid rows, bias param
__host__ __device__ constexpr int fwd_out_weight(int L, int n) {
  return L <= L7 ? 2 * L : L == LFA ? (n < 8 ? (int)P_FW : (int)P_AW) : L == LV ? (int)P_VW : (int)P_RW;
}
__host__ __device__ constexpr int fwd_out_row0(int L, int n) { return (L == LFA && n == 8) ? 0 : 32 * n; }
__host__ __device__ constexpr int fwd_out_valid(int L, int n) {
  return (L == LFA && n == 8) ? 1 : L == LRGB ? 3 : 32;
}

// forward units: one per (layer, output tile), in execution order
constexpr int NUNIT_FWD = 8 * 8 + 9 + 4 + 1;  // 78
__host__ __device__ constexpr int fwd_unit_first(int L) {
  int u = 0;
  for (int k = 0; k < L; ++k) u += fwd_out_tiles(k);
  return u;
}
__host__ __device__ constexpr int fwd_unit_layer(int u) {
  int L = 0;
  while (L < NLAYER - 1 && u >= fwd_unit_first(L + 1)) ++L;
  return L;
}
__host__ __device__ constexpr int fwd_unit_tiles(int u) { return fwd_in_tiles(fwd_unit_layer(u)); }
__host__ __device__ constexpr int fwd_unit_tile_off(int u) {  // in input tiles
  int o = 0;
  for (int k = 0; k < u; ++k) o += fwd_unit_tiles(k);
  return o;
}
constexpr int FWD_TILES = fwd_unit_tile_off(NUNIT_FWD);  // 592

// backward (dX chain) units, W^T products, in execution order:
//   bRGB (4 out tiles: hv), bV (8: feature), bFA (8: h7), b7, b6, b5 (-> h4), b4, b3, b2, b1 (-> h0)
enum BStage { B_RGB = 0, B_V, B_FA, B_7, B_6, B_5, B_4, B_3, B_2, B_1, NBSTAGE };
__host__ __device__ constexpr int bwd_fwd_layer(int s) {
  return s == B_RGB ? LRGB : s == B_V ? LV : s == B_FA ? LFA : (L7 - (s - B_7));
}
__host__ __device__ constexpr int bwd_out_tiles(int s) { return s == B_RGB ? 4 : 8; }
__host__ __device__ constexpr int bwd_in_tiles(int s) { return fwd_out_tiles(bwd_fwd_layer(s)); }
// output tile j of stage s -> first column of the forward weight it reads
__host__ __device__ constexpr int bwd_out_colbase(int s, int j) {
  return bwd_fwd_layer(s) == L5 ? 63 + 32 * j : 32 * j;
}
constexpr int NUNIT_BWD = 4 + 8 * 9;  // 76
__host__ __device__ constexpr int bwd_unit_first(int s) {
  int u = 0;
  for (int k = 0; k < s; ++k) u += bwd_out_tiles(k);
  return u;
}
__host__ __device__ constexpr int bwd_unit_stage(int u) {
  int s = 0;
  while (s < NBSTAGE - 1 && u >= bwd_unit_first(s + 1)) ++s;
  return s;
}
__host__ __device__ constexpr int bwd_unit_tiles(int u) { return bwd_in_tiles(bwd_unit_stage(u)); }
__host__ __device__ constexpr int bwd_unit_tile_off(int u) {
  int o = 0;
  for (int k = 0; k < u; ++k) o += bwd_unit_tiles(k);
  return o;
}
constexpr int BWD_TILES = bwd_unit_tile_off(NUNIT_BWD);

// 16-row forward units (round 6: the bf16x3 forward on v_mfma_f32_16x16x32_bf16, 16 samples per
// wave, two waves per SIMD).  Unit = one 16-row output tile of one layer; its input is the same
// list of 32-feature K-blocks as the 32-row forward's input tiles.  B operand of K-block t: lane
// l = s + 16 g (sample s, lane group g) holds 8 features, element e -> feature 32 t + k16_feat(g, e);
// a 16x16 accumulator holds rows 4 g + {0..3} of sample s, so output tiles 2t and 2t + 1 ARE the
// next layer's K-block t (elements 0..3 and 4..7) in registers, the weights permuted to match.
__host__ __device__ constexpr int k16_feat(int g, int e) { return e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4); }
__host__ __device__ constexpr int fwd16_out_tiles(int L) {
  return L == LFA ? 17 : L == LV ? 8 : L == LRGB ? 1 : 16;  // (LFA: 16 feature tiles + the alpha row)
}
constexpr int NUNIT_FWD16 = 8 * 16 + 17 + 8 + 1;  // 154
__host__ __device__ constexpr int fwd16_unit_first(int L) {
  int u = 0;
  for (int k = 0; k < L; ++k) u += fwd16_out_tiles(k);
  return u;
}
__host__ __device__ constexpr int fwd16_unit_layer(int u) {
  int L = 0;
  while (L < NLAYER - 1 && u >= fwd16_unit_first(L + 1)) ++L;
  return L;
}
__host__ __device__ constexpr int fwd16_unit_tiles(int u) { return fwd_in_tiles(fwd16_unit_layer(u)); }
__host__ __device__ constexpr int fwd16_unit_tile_off(int u) {  // in input K-blocks
  int o = 0;
  for (int k = 0; k < u; ++k) o += fwd16_unit_tiles(k);
  return o;
}
constexpr int FWD16_TILES = fwd16_unit_tile_off(NUNIT_FWD16);
// output tile m of layer L -> weight param, first weight row, valid rows
__host__ __device__ constexpr int fwd16_out_weight(int L, int m) {
  return L <= L7 ? 2 * L : L == LFA ? (m < 16 ? (int)P_FW : (int)P_AW) : L == LV ? (int)P_VW : (int)P_RW;
}
__host__ __device__ constexpr int fwd16_out_row0(int L, int m) { return (L == LFA && m == 16) ? 0 : 16 * m; }
__host__ __device__ constexpr int fwd16_out_valid(int L, int m) {
  return (L == LFA && m == 16) ? 1 : L == LRGB ? 3 : 16;
}
// 16-row dX units (round 6: the wide dX of PF32W / PBF3W): unit = one 16-row half m & 1 of output tile m >> 1 of a
// dX stage; its input is the stage's list of 32-feature K-blocks, in the same permuted order (k16_feat)
__host__ __device__ constexpr int bwd16_out_tiles(int s) { return 2 * bwd_out_tiles(s); }
constexpr int NUNIT_BWD16 = 8 + 16 * 9;  // 152
__host__ __device__ constexpr int bwd16_unit_first(int s) {
  int u = 0;
  for (int k = 0; k < s; ++k) u += bwd16_out_tiles(k);
  return u;
}
__host__ __device__ constexpr int bwd16_unit_stage(int u) {
  int s = 0;
  while (s < NBSTAGE - 1 && u >= bwd16_unit_first(s + 1)) ++s;
  return s;
}
__host__ __device__ constexpr int bwd16_unit_tiles(int u) { return bwd_in_tiles(bwd16_unit_stage(u)); }
__host__ __device__ constexpr int bwd16_unit_tile_off(int u) {
  int o = 0;
  for (int k = 0; k < u; ++k) o += bwd16_unit_tiles(k);
  return o;
}
constexpr int BWD16_TILES = bwd16_unit_tile_off(NUNIT_BWD16);

constexpr int NUNIT_MAX = NUNIT_FWD16;  // the largest unit table (forward 78, dX 76, 16-row forward 154, dX 152)
static_assert(NUNIT_FWD16 > NUNIT_FWD && NUNIT_FWD16 > NUNIT_BWD && NUNIT_FWD16 >= NUNIT_BWD16, "NUNIT_MAX");

// Training stores, "fragment-native": a stored tensor is a list of 32-feature tiles; tile
// tau of 32-sample block b occupies one tile-block of CH KiB at ((tau * nblk + b) * CH + c)
// KiB (chunk c = accumulator registers [c*E, c*E+E) of every lane, lane-linear, 16 B per
// lane) -- exactly the B-operand registers, so a wave stores a finished tile with CH
// 16-byte stores per lane.  The dW GEMM reads them back transposed (ds_read_b64_tr_b16).
enum ActTile {
  AT_X = 0,    // PE(xyz): 2 tiles (63 features + 1 zero)
  AT_D = 2,    // PE(dir): 1 tile (27 + 5 zero)
  AT_H = 3,    // h0..h7 post-ReLU: tile 3 + 8 l + n
  AT_F = 67,   // feature (no activation): 8 tiles
  AT_V = 75,   // views hidden post-ReLU: 4 tiles
  AT_TILES = 79
};
enum DzTile {
  ZT_H = 0,     // dZ0..dZ7 (pre-ReLU grads of pts_linears): tile 8 l + n
  ZT_F = 64,    // d feature: 8
  ZT_A = 72,    // d alpha: row 0 of one tile
  ZT_V = 73,    // dZ views: 4
  ZT_RGB = 77,  // d rgb: rows 0..2 of one tile
  ZT_TILES = 78
};
constexpr int A_ROWS = AT_TILES * 32;  // 2528 feature rows
constexpr int Z_ROWS = ZT_TILES * 32;  // 2496
// ReLU masks: per 32-sample wave block, 9 groups x 64 lanes x 16 B (layers h0..h7: 8 tiles x
// 16 bits each; group 8: the 4 view-layer tiles)
constexpr int MASK_GROUPS = 9;

// dW GEMM list (per net): C[n][k] = sum_m dz[n][m] act[k][m]
constexpr int NGEMM = 12;
__host__ __device__ constexpr int gemm_weight(int g) {
  return g < 8 ? 2 * g : g == 8 ? (int)P_FW : g == 9 ? (int)P_AW : g == 10 ? (int)P_VW : (int)P_RW;
}
__host__ __device__ constexpr int gemm_dz_tile(int g, int nt) {
  return g < 8 ? ZT_H + 8 * g + nt : g == 8 ? ZT_F + nt : g == 9 ? (int)ZT_A : g == 10 ? ZT_V + nt : (int)ZT_RGB;
}
__host__ __device__ constexpr int gemm_n_tiles(int g) { return g < 9 ? 8 : g == 9 ? 1 : g == 10 ? 4 : 1; }
__host__ __device__ constexpr int gemm_n_valid(int g) { return g == 9 ? 1 : g == 11 ? 3 : (g == 10 ? 128 : 256); }
__host__ __device__ constexpr int gemm_k_tiles(int g) {
  return g == 0 ? 2 : g == 5 ? 10 : g == 10 ? 9 : g == 11 ? 4 : 8;
}
// k tile t of gemm g -> (act tile, first weight column, valid columns)
__host__ __device__ constexpr int gemm_act_tile(int g, int t) {
  return g == 0 ? AT_X + t
       : g == 5 ? (t < 2 ? AT_X + t : AT_H + 8 * 4 + (t - 2))
       : g <= 7 ? AT_H + 8 * (g - 1) + t
       : g <= 9 ? AT_H + 8 * 7 + t
       : g == 10 ? (t < 8 ? AT_F + t : (int)AT_D)
       : AT_V + t;
}
__host__ __device__ constexpr int gemm_col0(int g, int t) {
  return g == 0 ? 32 * t : g == 5 ? (t < 2 ? 32 * t : 63 + 32 * (t - 2)) : 32 * t;
}
__host__ __device__ constexpr int gemm_col_valid(int g, int t) {
  return (g == 0 || g == 5) && t == 1 ? 31 : (g == 10 && t == 8) ? 27 : 32;
}

}  // namespace mlp
}  // namespace nerf
