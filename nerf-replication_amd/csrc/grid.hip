// Occupancy grid on gfx950: cell lookup, baking (grid update) and the grid-accelerated
// ray march with early ray termination.
//
// Reference semantics (echo636/nerf-replication):
//   world_to_grid_indices   src/models/nerf/renderer/volume_renderer.py:261-265
//   render_accelerated      volume_renderer.py:268-357
//   grid bake               occupancy_grid.py:15-80
//
// The reference marches all alive rays one t-step at a time (800 Python iterations, a
// host sync each).  Here each round lets every alive ray collect its next K occupied
// steps (gather), the fine MLP runs once on all collected points, and a per-ray
// compositor consumes them in t order, stopping exactly where the reference would
// (T < threshold after a queried step).  Points past a ray's termination are evaluated
// but never composited, so outputs are those of the step-by-step march.
#include "common.h"

namespace nerf {

struct BBox { float mn[3], mx[3]; };

__device__ __forceinline__ int grid_axis(float p, float mn, float mx, int res) {
  const float c = fminf(fmaxf(p, mn), mx);                  // torch.clamp(p, min, max)
  const float n = fdiv(fsub(c, mn), fsub(mx, mn));          // (p - min) / (max - min)
  return (int)fmul(n, (float)(res - 1));                    // (n * (res - 1)).long()
}

struct GridIndexArgs {
  const float* pts;
  int64_t M;
  BBox bb;
  int res;
  const uint8_t* grid;
  int64_t* idx;
  uint8_t* occ;
};

__global__ void grid_index_kernel(GridIndexArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.M) return;
  int ix = grid_axis(a.pts[i * 3 + 0], a.bb.mn[0], a.bb.mx[0], a.res);
  int iy = grid_axis(a.pts[i * 3 + 1], a.bb.mn[1], a.bb.mx[1], a.res);
  int iz = grid_axis(a.pts[i * 3 + 2], a.bb.mn[2], a.bb.mx[2], a.res);
  if (a.idx) {
    a.idx[i * 3 + 0] = ix;
    a.idx[i * 3 + 1] = iy;
    a.idx[i * 3 + 2] = iz;
  }
  if (a.occ) a.occ[i] = a.grid[((int64_t)ix * a.res + iy) * a.res + iz];
}

// ------------------------------------------------------------------------------------
// bake
// ------------------------------------------------------------------------------------
// A bake covers the voxel slab x in [x0, x1) (the whole grid: [0, res)); point and grid
// indices are slab-relative.
struct BakeArgs {
  int res;
  BBox bb;
  int dedup;   // 1: (x1-x0+1)(res+1)^2 lattice points; 0: (x1-x0) res^2 x 8 corners
  int x0, x1;
  float* pts;
};

__device__ __forceinline__ float voxel_size(const BBox& bb, int k, int res) {
  return fdiv(fsub(bb.mx[k], bb.mn[k]), (float)res);
}

__global__ void bake_points_kernel(BakeArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nx = a.x1 - a.x0;
  if (a.dedup) {
    const int64_t n = (int64_t)(a.res + 1);
    if (i >= (nx + 1) * n * n) return;
    const int L[3] = {a.x0 + (int)(i / (n * n)), (int)((i / n) % n), (int)(i % n)};
#pragma unroll
    for (int k = 0; k < 3; ++k)
      a.pts[i * 3 + k] = fadd(a.bb.mn[k], fmul((float)L[k], voxel_size(a.bb, k, a.res)));
  } else {
    const int64_t n = (int64_t)a.res;
    if (i >= nx * n * n * 8) return;
    const int64_t v = i >> 3;
    const int c = (int)(i & 7);  // meshgrid 'ij' over the 2x2x2 corner offsets
    const int idx[3] = {a.x0 + (int)(v / (n * n)), (int)((v / n) % n), (int)(v % n)};
    const int off[3] = {(c >> 2) & 1, (c >> 1) & 1, c & 1};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float vs = voxel_size(a.bb, k, a.res);
      const float base = fadd(a.bb.mn[k], fmul((float)idx[k], vs));
      a.pts[i * 3 + k] = fadd(base, off[k] ? vs : 0.f);
    }
  }
}

struct BakeReduceArgs {
  const float* raw;  // [P,4] (slab points)
  int res, dedup;
  int x0, x1;
  float threshold;
  uint8_t* grid;     // [x1 - x0][res][res]
};

__global__ void bake_reduce_kernel(BakeReduceArgs a) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = a.res;
  if (v >= (int64_t)(a.x1 - a.x0) * n * n) return;
  const int x = (int)(v / (n * n)), y = (int)((v / n) % n), z = (int)(v % n);
  bool occ = false;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    int64_t p;
    if (a.dedup) {
      const int64_t m = n + 1;
      p = ((int64_t)(x + ((c >> 2) & 1)) * m + (y + ((c >> 1) & 1))) * m + (z + (c & 1));
    } else {
      p = v * 8 + c;
    }
    const float s = a.raw[p * 4 + 3];
    const float sigma = s > 0.f ? s : 0.f;  // relu(raw[..., 3])
    occ |= sigma > a.threshold;
  }
  a.grid[v] = occ ? 1 : 0;
}

// ------------------------------------------------------------------------------------
// march
// ------------------------------------------------------------------------------------
struct MarchState {
  float* T;
  float* rgb;
  float* depth;
  float* acc;
  int32_t* next_step;
  uint8_t* alive;     // 1 = still marching
  uint8_t* exhausted; // 1 = gather reached the end of the t table
};

struct MarchGatherArgs {
  const float* rays;  // [N,6]
  int64_t N;
  const float* t_table;
  int n_steps;
  const uint8_t* grid;
  int res;
  const uint8_t* macro;  // [mres^3] 1 = some cell of the 8^3 block occupied (nerf_march_macro), or null
  BBox bb;
  int K;
  int k_low;       // rays with T < t_split gather at most k_low steps (they terminate soon)
  float t_split;
  MarchState st;
  int32_t* counters;   // [0] points reserved, [1] rays alive entering the round
  unsigned long long* evaluated;  // += points written below cap (what the MLP evaluates), or null
  int32_t* out_ray;    // [cap]
  int32_t* out_step;   // [cap]
  float* out_pts;      // [cap,3]
  int32_t* ray_off;    // [N]
  int32_t* ray_cnt;    // [N]
  int64_t cap;
};

__device__ __forceinline__ bool march_occupied(const MarchGatherArgs& a, const float* ray, float t, float* p,
                                               int* cell) {
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = fadd(ray[k], fmul(t, ray[3 + k]));  // o + t * d
#pragma unroll
  for (int k = 0; k < 3; ++k) cell[k] = grid_axis(p[k], a.bb.mn[k], a.bb.mx[k], a.res);
  return a.grid[((int64_t)cell[0] * a.res + cell[1]) * a.res + cell[2]] != 0;
}

// Empty-cell skip (exact).  The step walk is latency-bound (one dependent grid lookup per
// 0.005 step, ~4.7 steps per cell).  After an EMPTY cell, the steps that provably map to the
// same cell are skipped: along each axis the cell index is a monotone function of p (clamp,
// subtract, divide, multiply, truncate: each monotone in fp32), so its preimage is an interval
// [lo, hi) -- within a few ulps of mn + i w, w = (mx - mn) / (res - 1), open-ended for the
// boundary cells that also hold the clamped outside -- and the computed p = o + t d is monotone
// in t.  Every step whose t is below the first exit of the interval SHRUNK by a margin m is
// therefore in the same empty cell, and is skipped; the walk resumes one step at a time near the
// boundary.  m = max(1e-3 w, 2^-18 (|o| + t_abs |d| + |mn| + |mx|)), t_abs = max(8, |t| over the
// table) (a far bound past 8 widens the margin with the coordinates): 1e-3 w is ~2.4e-5 at res 128, but
// shrinks as 1/res (2.9e-6 at res 1024), while the fp32 errors of p = o + t d, of the interval
// bounds and of t_exit d are a few ulps of the coordinates' magnitude (~1e-6 for |o| ~ 4, t <= 6
// here): the absolute floor keeps the margin >= 8 such ulps at any resolution.  Returns the next
// step to test (> s).
//
// Two levels: when the whole 8^3 block of cells around an empty cell is empty (the macro grid,
// nerf_march_macro), the interval is the block's -- cells [8 j, 8 j + 7] along each axis, the
// same monotone argument over a union of cells -- so a ray crosses empty space ~8x faster (the
// walk is a chain of dependent lookups: its length, not the lookups, sets a round's gather time).
constexpr int MACRO = 8;
__device__ __forceinline__ int march_skip_empty(const MarchGatherArgs& a, const float* ray, int s, const int* cell,
                                                int span) {
  // fp32 with approximate reciprocals: the errors (~1e-6 in p) are far inside the margin.
  // |t| is bounded by the table's ends (it is monotone); 8 is the floor the bound was tested at
  const float t_abs = fmaxf(8.0f, fmaxf(fabsf(a.t_table[0]), fabsf(a.t_table[a.n_steps - 1])));
  float t_exit = 3.0e38f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float d = ray[3 + k];
    const float mn = a.bb.mn[k], w = (a.bb.mx[k] - mn) * (1.0f / (float)(a.res - 1));
    const float mag = fabsf(ray[k]) + t_abs * fabsf(d) + fabsf(mn) + fabsf(a.bb.mx[k]);
    const float m = fmaxf(1e-3f * w, mag * 3.814697265625e-6f);  // 2^-18
    const int lo = cell[k] / span * span, hi = min(lo + span - 1, a.res - 1);  // the interval's cells
    const float rd = __builtin_amdgcn_rcpf(d);
    if (d > 0.0f && hi < a.res - 1) {         // (at max, clamped: stays while p grows)
      t_exit = fminf(t_exit, (mn + (float)(hi + 1) * w - m - ray[k]) * rd);
    } else if (d < 0.0f && lo > 0) {          // (at min, clamped: stays while p falls)
      t_exit = fminf(t_exit, (mn + (float)lo * w + m - ray[k]) * rd);
    }
  }
  // last step j > s with t_table[j] < t_exit (steps are ~uniform: estimate, then correct)
  const float t0 = a.t_table[s], t1 = a.t_table[a.n_steps > s + 1 ? s + 1 : s];
  int j = s;
  if (t1 > t0 && t_exit > t1) {
    const float est = (t_exit - t0) * __builtin_amdgcn_rcpf(t1 - t0);
    j = s + (int)fminf(est, (float)(a.n_steps - 1 - s)) - 1;
    if (j < s) j = s;
    while (j + 1 < a.n_steps && a.t_table[j + 1] < t_exit) ++j;
    while (j > s && a.t_table[j] >= t_exit) --j;
  }
  return j + 1;
}

// the step after an empty cell: the macro block's exit when the block is empty, else the cell's
__device__ __forceinline__ int march_next_after_empty(const MarchGatherArgs& a, const float* ray, int s,
                                                      const int* cell) {
  int span = 1;
  if (a.macro) {
    const int mres = (a.res + MACRO - 1) / MACRO;
    const int64_t j = ((int64_t)(cell[0] / MACRO) * mres + cell[1] / MACRO) * mres + cell[2] / MACRO;
    if (a.macro[j] == 0) span = MACRO;
  }
  return march_skip_empty(a, ray, s, cell, span);
}

__global__ void march_gather_kernel(MarchGatherArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = r < a.N;
  const bool live = in && a.st.alive[r];
  int cnt = 0, s = live ? a.st.next_step[r] : 0;
  const float* ray = a.rays + (in ? r : 0) * 6;
  float p[3];
  if (live) {
    // a ray whose transmittance has already dropped is near its termination step: gathering
    // few steps for it wastes fewer speculative MLP evaluations (outputs are unchanged -- the
    // compositor stops where the reference does, and an unfinished ray gathers again)
    const int k = a.st.T[r] < a.t_split ? (a.k_low < a.K ? a.k_low : a.K) : a.K;
    int cell[3];
    while (s < a.n_steps && cnt < k) {
      if (march_occupied(a, ray, a.t_table[s], p, cell)) {
        ++cnt;
        ++s;
      } else {
        s = march_next_after_empty(a, ray, s, cell);
      }
    }
  }
  // wave-aggregated reservation
  const int l = lane_id();
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(incl, o, 64);
    if (l >= o) incl += t;
  }
  const int wtotal = __shfl(incl, 63, 64);
  int base = 0;
  if (l == 63 && wtotal > 0) {
    base = atomicAdd(&a.counters[0], wtotal);
    // the positions of this wave's reservation below cap are all written (by emit)
    const int64_t below = a.cap - (int64_t)base;
    if (a.evaluated && below > 0) atomicAdd(a.evaluated, (unsigned long long)(below < wtotal ? below : wtotal));
  }
  base = __shfl(base, 63, 64);
  const unsigned long long live_mask = __ballot(live);
  if (l == 0 && live_mask) atomicAdd(&a.counters[1], __popcll(live_mask));
  if (!in) return;
  if (!live) {
    a.ray_cnt[r] = 0;
    return;
  }
  int pos = base + incl - cnt;
  const bool overflow = (int64_t)pos + cnt > a.cap;
  a.ray_off[r] = pos;
  // out of room: the ray keeps its position and gathers again next round.  The part of its
  // reservation below cap is still written by emit (ray_cnt = -that many: not composited), so
  // that every position below min(points reserved, cap) holds a valid point and ray id -- the
  // MLP launch sized on the device (nerf_mlp_fwd_count) reads exactly that prefix.
  if (overflow) {
    const int64_t room = a.cap - (int64_t)pos;
    a.ray_cnt[r] = -(int)(room <= 0 ? 0 : room < cnt ? room : cnt);
    return;
  }
  a.ray_cnt[r] = cnt;
  a.st.exhausted[r] = (s >= a.n_steps) ? 1 : 0;
  a.st.next_step[r] = s;
}

// Two-pass variant that keeps the start step: the gather kernel above records counts;
// this kernel writes the points.
struct MarchEmitArgs {
  MarchGatherArgs g;
  const int32_t* start_step;  // [N] step before the gather
};

__global__ void march_emit_kernel(MarchEmitArgs e) {
  const MarchGatherArgs& a = e.g;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.N) return;
  const int c = a.ray_cnt[r];
  const int cnt = c < 0 ? -c : c;  // (< 0: an overflowing ray's points below cap, written only)
  if (cnt == 0) return;
  const float* ray = a.rays + r * 6;
  int pos = a.ray_off[r];
  int k = 0;
  float p[3];
  int cell[3];
  for (int s = e.start_step[r]; k < cnt;) {  // the gather's walk, skips included
    if (march_occupied(a, ray, a.t_table[s], p, cell)) {
      a.out_ray[pos + k] = (int32_t)r;
      a.out_step[pos + k] = s;
      a.out_pts[(int64_t)(pos + k) * 3 + 0] = p[0];
      a.out_pts[(int64_t)(pos + k) * 3 + 1] = p[1];
      a.out_pts[(int64_t)(pos + k) * 3 + 2] = p[2];
      ++k;
      ++s;
    } else {
      s = march_next_after_empty(a, ray, s, cell);
    }
  }
}

// One-pass gather + emit (the default since round 3).  The two-pass form above walks every
// ray twice: once to count its points (the wave's reservation needs every lane's count
// first), once more, with every grid lookup again, to write them (the bf16 trained-net frame:
// 1.4 of 17 ms in emit).  Here the counting walk records where the points are -- as runs of
// consecutive occupied steps, up to MARCH_RUNS per lane in LDS (a run of an occupied cell is
// ~4.7 steps) plus the open one in registers -- and the points are written from the runs
// after the reservation, with no lookups.  A lane whose runs do not fit remembers where its
// first unrecorded run starts and walks again from there for the rest (the same walk: the
// same steps).  Outputs, counters and overflow handling are those of gather + emit.
constexpr int MARCH_RUNS = 16;
constexpr int MARCH_WAVES = 4;  // 256-thread blocks
__device__ __forceinline__ void march_put(const MarchGatherArgs& a, int64_t r, const float* ray, int64_t at, int s) {
  float p[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = fadd(ray[k], fmul(a.t_table[s], ray[3 + k]));  // = march_occupied's p
  a.out_ray[at] = (int32_t)r;
  a.out_step[at] = s;
  a.out_pts[at * 3 + 0] = p[0];
  a.out_pts[at * 3 + 1] = p[1];
  a.out_pts[at * 3 + 2] = p[2];
}

__global__ void __launch_bounds__(256) march_gather_emit_kernel(MarchGatherArgs a) {
  __shared__ uint32_t runs[MARCH_WAVES][MARCH_RUNS][64];  // (start << 16) | length, lane-minor
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int w = threadIdx.x >> 6, l = lane_id();
  const bool in = r < a.N;
  const bool live = in && a.st.alive[r];
  int cnt = 0, s = live ? a.st.next_step[r] : 0;
  const float* ray = a.rays + (in ? r : 0) * 6;
  int nrun = 0, cur_start = 0, cur_len = 0;  // recorded runs; the open run
  int ovf_step = -1;                           // first unrecorded run's step
  if (live) {
    const int k = a.st.T[r] < a.t_split ? (a.k_low < a.K ? a.k_low : a.K) : a.K;
    float p[3];
    int cell[3];
    while (s < a.n_steps && cnt < k) {
      if (march_occupied(a, ray, a.t_table[s], p, cell)) {
        if (ovf_step < 0) {
          if (cur_len > 0 && s == cur_start + cur_len && cur_len < 0xFFFF) {
            ++cur_len;
          } else {
            if (cur_len > 0) {
              if (nrun < MARCH_RUNS) {
                runs[w][nrun][l] = ((uint32_t)cur_start << 16) | (uint32_t)cur_len;
                ++nrun;
              } else {  // out of slots: the open run and everything after it are walked again
                ovf_step = cur_start;
              }
            }
            if (ovf_step < 0) {
              cur_start = s;
              cur_len = 1;
            }
          }
        }
        ++cnt;
        ++s;
      } else {
        s = march_next_after_empty(a, ray, s, cell);
      }
    }
  }
  // wave-aggregated reservation (as march_gather_kernel)
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(incl, o, 64);
    if (l >= o) incl += t;
  }
  const int wtotal = __shfl(incl, 63, 64);
  int base = 0;
  if (l == 63 && wtotal > 0) {
    base = atomicAdd(&a.counters[0], wtotal);
    const int64_t below = a.cap - (int64_t)base;
    if (a.evaluated && below > 0) atomicAdd(a.evaluated, (unsigned long long)(below < wtotal ? below : wtotal));
  }
  base = __shfl(base, 63, 64);
  const unsigned long long live_mask = __ballot(live);
  if (l == 0 && live_mask) atomicAdd(&a.counters[1], __popcll(live_mask));
  if (!in) return;
  if (!live) {
    a.ray_cnt[r] = 0;
    return;
  }
  const int pos = base + incl - cnt;
  const bool overflow = (int64_t)pos + cnt > a.cap;
  a.ray_off[r] = pos;
  int nwrite = cnt;
  if (overflow) {  // out of room: written below cap only, gathered again next round
    const int64_t room = a.cap - (int64_t)pos;
    nwrite = (int)(room <= 0 ? 0 : room < cnt ? room : cnt);
    a.ray_cnt[r] = -nwrite;
  } else {
    a.ray_cnt[r] = cnt;
    a.st.exhausted[r] = (s >= a.n_steps) ? 1 : 0;
    a.st.next_step[r] = s;
  }
  // emit: the recorded runs, the open run, then (after a run overflow) the walk again
  int kk = 0;
  for (int i = 0; i < nrun && kk < nwrite; ++i) {
    const uint32_t ru = runs[w][i][l];
    const int st = (int)(ru >> 16), ln = (int)(ru & 0xFFFF);
    for (int j = 0; j < ln && kk < nwrite; ++j, ++kk) march_put(a, r, ray, (int64_t)pos + kk, st + j);
  }
  if (ovf_step < 0) {
    for (int j = 0; j < cur_len && kk < nwrite; ++j, ++kk) march_put(a, r, ray, (int64_t)pos + kk, cur_start + j);
  } else {
    float p[3];
    int cell[3];
    for (int ss = ovf_step; kk < nwrite;) {
      if (march_occupied(a, ray, a.t_table[ss], p, cell)) {
        march_put(a, r, ray, (int64_t)pos + kk, ss);
        ++kk;
        ++ss;
      } else {
        ss = march_next_after_empty(a, ray, ss, cell);
      }
    }
  }
}

struct MarchCompArgs {
  const float* raw;  // [cap,4]
  const float* rays;
  int64_t N;
  const float* t_table;
  const int32_t* ray_off;
  const int32_t* ray_cnt;
  const int32_t* out_step;
  MarchState st;
  float step_size, t_thresh;
  unsigned long long* consumed;  // += points composited (the reference's MLP queries) or null
};

__device__ __forceinline__ int march_composite_ray_impl(const MarchCompArgs& a, int64_t r);
__device__ __forceinline__ int march_composite_ray(const MarchCompArgs& a, int64_t r) {
  return march_composite_ray_impl(a, r);
}

// Composites a ray's gathered points in step order and stops at T < t_thresh
// (volume_renderer.py:327-341).  Points gathered past that step were evaluated speculatively
// and are dropped; the points composited are exactly the reference's queries (:324), counted
// into `consumed`.
__global__ void march_composite_kernel(MarchCompArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = r < a.N && a.st.alive[r];
  int used = 0;
  if (live) used = march_composite_ray(a, r);
  if (a.consumed) {
    // wave-aggregated count
    int tot = used;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
    if (lane_id() == 0 && tot) atomicAdd(a.consumed, (unsigned long long)tot);
  }
}

__device__ __forceinline__ int march_composite_ray_impl(const MarchCompArgs& a, int64_t r) {
  const int c = a.ray_cnt[r], off = a.ray_off[r];
  const int cnt = c > 0 ? c : 0;  // (< 0: gathered nothing this round, see march_gather_kernel)
  const float* ray = a.rays + r * 6;
  const float dx = ray[3], dy = ray[4], dz = ray[5];
  const float dist = fmul(a.step_size, sqrtf(fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz))));
  float T = a.st.T[r];
  float cr = a.st.rgb[r * 3 + 0], cg = a.st.rgb[r * 3 + 1], cb = a.st.rgb[r * 3 + 2];
  float dep = a.st.depth[r], acc = a.st.acc[r];
  bool alive = true;
  int used = cnt;
  for (int k = 0; k < cnt; ++k) {
    const float4 rw = *(const float4*)(a.raw + (int64_t)(off + k) * 4);
    const float t = a.t_table[a.out_step[off + k]];
    const float sr = 1.f / (1.f + expf(-rw.x)), sg = 1.f / (1.f + expf(-rw.y)), sb = 1.f / (1.f + expf(-rw.z));
    const float sigma = rw.w > 0.f ? rw.w : 0.f;
    const float alpha = fsub(1.f, expf(-fmul(sigma, dist)));
    const float ta = fmul(T, alpha);
    cr = fadd(cr, fmul(ta, sr));
    cg = fadd(cg, fmul(ta, sg));
    cb = fadd(cb, fmul(ta, sb));
    acc = fadd(acc, ta);
    dep = fadd(dep, fmul(ta, t));
    T = fmul(T, fsub(1.f, alpha));
    if (T < a.t_thresh) {
      alive = false;
      used = k + 1;
      break;
    }
  }
  a.st.T[r] = T;
  a.st.rgb[r * 3 + 0] = cr;
  a.st.rgb[r * 3 + 1] = cg;
  a.st.rgb[r * 3 + 2] = cb;
  a.st.depth[r] = dep;
  a.st.acc[r] = acc;
  if (!alive || a.st.exhausted[r]) a.st.alive[r] = 0;
  return used;
}

// macro occupancy: block (i, j, k) = cells [8 i, 8 i + 8) x [8 j, ..) x [8 k, ..) (clipped at res)
__global__ void march_macro_kernel(const uint8_t* grid, int res, uint8_t* macro) {
  const int mres = (res + MACRO - 1) / MACRO;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= (int64_t)mres * mres * mres) return;
  const int bi = (int)(b / ((int64_t)mres * mres)), bj = (int)((b / mres) % mres), bk = (int)(b % mres);
  uint8_t any = 0;
  for (int i = bi * MACRO; i < min(bi * MACRO + MACRO, res); ++i)
    for (int j = bj * MACRO; j < min(bj * MACRO + MACRO, res); ++j)
      for (int k = bk * MACRO; k < min(bk * MACRO + MACRO, res); ++k) any |= grid[((int64_t)i * res + j) * res + k];
  macro[b] = any ? 1 : 0;
}

struct MarchInitArgs { MarchState st; int64_t N; };
__global__ void march_init_kernel(MarchInitArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.N) return;
  a.st.T[r] = 1.f;
  a.st.rgb[r * 3 + 0] = a.st.rgb[r * 3 + 1] = a.st.rgb[r * 3 + 2] = 0.f;
  a.st.depth[r] = 0.f;
  a.st.acc[r] = 0.f;
  a.st.next_step[r] = 0;
  a.st.alive[r] = 1;
  a.st.exhausted[r] = 0;
}

struct MarchFinishArgs { MarchState st; int64_t N; int white; };
__global__ void march_finish_kernel(MarchFinishArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.N || !a.white) return;
  const float bg = fsub(1.f, a.st.acc[r]);  // rgb += (1 - acc) * 1
#pragma unroll
  for (int k = 0; k < 3; ++k) a.st.rgb[r * 3 + k] = fadd(a.st.rgb[r * 3 + k], bg);
}

}  // namespace nerf

// ======================================================================================
// C-ABI
// ======================================================================================
using namespace nerf;

static BBox make_bbox(const float* b) {
  BBox bb;
  for (int k = 0; k < 3; ++k) {
    bb.mn[k] = b[k];
    bb.mx[k] = b[3 + k];
  }
  return bb;
}

static inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

extern "C" {

int nerf_grid_index(const float* pts, int64_t M, const float* bbox_host, int res, const uint8_t* grid,
                    int64_t* idx_out, uint8_t* occ_out, hipStream_t stream) {
  NERF_REQUIRE(M >= 0 && res > 1 && bbox_host, "nerf_grid_index: bad arguments");
  if (M == 0) return 0;
  NERF_REQUIRE(pts && (idx_out || occ_out), "nerf_grid_index: null pointer");
  NERF_REQUIRE(!occ_out || grid, "nerf_grid_index: occupancy needs the grid");
  GridIndexArgs a{pts, M, make_bbox(bbox_host), res, grid, idx_out, occ_out};
  hipLaunchKernelGGL(grid_index_kernel, grid1(M), dim3(256), 0, stream, a);
  return check_launch("nerf_grid_index");
}

int64_t nerf_bake_num_points_slab(int res, int dedup, int x0, int x1) {
  const int64_t n = res, nx = x1 - x0;
  if (res <= 0 || x0 < 0 || x1 > res || nx < 0) return -1;
  if (nx == 0) return 0;
  return dedup ? (nx + 1) * (n + 1) * (n + 1) : nx * n * n * 8;
}
int64_t nerf_bake_num_points(int res, int dedup) { return nerf_bake_num_points_slab(res, dedup, 0, res); }

int nerf_bake_points_slab(int res, const float* bbox_host, int dedup, int x0, int x1, float* pts,
                          hipStream_t stream) {
  NERF_REQUIRE(res > 0 && bbox_host && 0 <= x0 && x0 <= x1 && x1 <= res, "nerf_bake_points: bad arguments");
  if (x0 == x1) return 0;
  NERF_REQUIRE(pts, "nerf_bake_points: null pointer");
  BakeArgs a{res, make_bbox(bbox_host), dedup, x0, x1, pts};
  hipLaunchKernelGGL(bake_points_kernel, grid1(nerf_bake_num_points_slab(res, dedup, x0, x1)), dim3(256), 0, stream,
                     a);
  return check_launch("nerf_bake_points");
}
int nerf_bake_points(int res, const float* bbox_host, int dedup, float* pts, hipStream_t stream) {
  return nerf_bake_points_slab(res, bbox_host, dedup, 0, res, pts, stream);
}

int nerf_bake_reduce_slab(const float* raw, int res, int dedup, int x0, int x1, float threshold, uint8_t* grid,
                          hipStream_t stream) {
  NERF_REQUIRE(res > 0 && 0 <= x0 && x0 <= x1 && x1 <= res, "nerf_bake_reduce: bad arguments");
  if (x0 == x1) return 0;
  NERF_REQUIRE(raw && grid, "nerf_bake_reduce: null pointer");
  BakeReduceArgs a{raw, res, dedup, x0, x1, threshold, grid};
  hipLaunchKernelGGL(bake_reduce_kernel, grid1((int64_t)(x1 - x0) * res * res), dim3(256), 0, stream, a);
  return check_launch("nerf_bake_reduce");
}
int nerf_bake_reduce(const float* raw, int res, int dedup, float threshold, uint8_t* grid, hipStream_t stream) {
  return nerf_bake_reduce_slab(raw, res, dedup, 0, res, threshold, grid, stream);
}

// state: T, rgb[3], depth, acc (f32) ; next_step (i32) ; alive, exhausted (u8)
int nerf_march_init(float* T, float* rgb, float* depth, float* acc, int32_t* next_step, uint8_t* alive,
                    uint8_t* exhausted, int64_t N, hipStream_t stream) {
  if (N == 0) return 0;
  NERF_REQUIRE(T && rgb && depth && acc && next_step && alive && exhausted, "nerf_march_init: null pointer");
  MarchInitArgs a{{T, rgb, depth, acc, next_step, alive, exhausted}, N};
  hipLaunchKernelGGL(march_init_kernel, grid1(N), dim3(256), 0, stream, a);
  return check_launch("nerf_march_init");
}

// counters[0] = points reserved, counters[1] = rays alive entering this round (zero them first);
// evaluated (nullable) += the points written, min(points reserved, cap).
// start_step_scratch: [N] int32 workspace of the two-pass form (gather, then emit walking again),
// or null: the one-pass form (march_gather_emit_kernel, the default).
int64_t nerf_march_macro_bytes(int res) {
  if (res <= 1) return -1;
  const int64_t m = (res + MACRO - 1) / MACRO;
  return m * m * m;
}

int nerf_march_macro(const uint8_t* grid, int res, uint8_t* macro, hipStream_t stream) {
  NERF_REQUIRE(res > 1, "nerf_march_macro: bad res");
  NERF_REQUIRE(grid && macro, "nerf_march_macro: null pointer");
  hipLaunchKernelGGL(march_macro_kernel, grid1(nerf_march_macro_bytes(res)), dim3(256), 0, stream, grid, res, macro);
  return check_launch("nerf_march_macro");
}

int nerf_march_gather(const float* rays, int64_t N, const float* t_table, int n_steps, const uint8_t* grid, int res,
                      const uint8_t* macro, const float* bbox_host, int K, int k_low, float t_split, float* T,
                      float* rgb, float* depth,
                      float* acc,
                      int32_t* next_step, uint8_t* alive, uint8_t* exhausted, int32_t* counters,
                      unsigned long long* evaluated, int32_t* start_step_scratch, int32_t* out_ray, int32_t* out_step,
                      float* out_pts, int32_t* ray_off, int32_t* ray_cnt, int64_t cap, hipStream_t stream) {
  NERF_REQUIRE(N >= 0 && n_steps >= 0 && K > 0 && res > 1 && bbox_host, "nerf_march_gather: bad arguments");
  NERF_REQUIRE(cap >= K && cap <= INT32_MAX, "nerf_march_gather: need K <= cap <= INT32_MAX (point offsets are int32)");
  if (N == 0) return 0;
  NERF_REQUIRE(k_low > 0, "nerf_march_gather: k_low must be > 0");
  MarchGatherArgs a{rays, N, t_table, n_steps, grid, res, macro, make_bbox(bbox_host), K, k_low, t_split,
                    {T, rgb, depth, acc, next_step, alive, exhausted},
                    counters, evaluated, out_ray, out_step, out_pts, ray_off, ray_cnt, cap};
  if (!start_step_scratch) {  // one pass: gather + emit fused (march_gather_emit_kernel)
    NERF_REQUIRE(n_steps < 65536, "nerf_march_gather: the one-pass form needs n_steps < 65536 (16-bit run starts)");
    hipLaunchKernelGGL(march_gather_emit_kernel, grid1(N), dim3(256), 0, stream, a);
    return check_launch("nerf_march_gather");
  }
  if (hipMemcpyAsync(start_step_scratch, next_step, N * sizeof(int32_t), hipMemcpyDeviceToDevice, stream) !=
      hipSuccess) {
    set_error("nerf_march_gather: hipMemcpyAsync failed");
    return -5;
  }
  hipLaunchKernelGGL(march_gather_kernel, grid1(N), dim3(256), 0, stream, a);
  if (int e = check_launch("nerf_march_gather")) return e;
  MarchEmitArgs em{a, start_step_scratch};
  hipLaunchKernelGGL(march_emit_kernel, grid1(N), dim3(256), 0, stream, em);
  return check_launch("nerf_march_emit");
}

int nerf_march_composite(const float* raw, const float* rays, int64_t N, const float* t_table, const int32_t* ray_off,
                         const int32_t* ray_cnt, const int32_t* out_step, float* T, float* rgb, float* depth,
                         float* acc, int32_t* next_step, uint8_t* alive, uint8_t* exhausted, float step_size,
                         float t_thresh, unsigned long long* consumed, hipStream_t stream) {
  if (N == 0) return 0;
  MarchCompArgs a{raw, rays, N, t_table, ray_off, ray_cnt, out_step,
                  {T, rgb, depth, acc, next_step, alive, exhausted}, step_size, t_thresh, consumed};
  hipLaunchKernelGGL(march_composite_kernel, grid1(N), dim3(256), 0, stream, a);
  return check_launch("nerf_march_composite");
}

int nerf_march_finish(float* rgb, const float* acc, int64_t N, int white, hipStream_t stream) {
  if (N == 0) return 0;
  MarchFinishArgs a{{nullptr, rgb, nullptr, const_cast<float*>(acc), nullptr, nullptr, nullptr}, N, white};
  hipLaunchKernelGGL(march_finish_kernel, grid1(N), dim3(256), 0, stream, a);
  return check_launch("nerf_march_finish");
}

}  // extern "C"
