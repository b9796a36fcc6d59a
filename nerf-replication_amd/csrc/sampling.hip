// Ray generation, stratified sampling, inverse-CDF importance sampling (+ merge) and
// alpha compositing (forward / backward) for the NeRF render-and-train path on gfx950.
//
// Reference semantics (echo636/nerf-replication):
//   raygen            src/datasets/nerf/blender.py:13-32 (get_rays), :124-131 (train batch)
//   stratified        src/models/nerf/renderer/volume_renderer.py:165-187
//   sample_pdf        volume_renderer.py:82-134, merge/sort :205-221
//   composite fwd     volume_renderer.py:20-80 (raw2outputs, raw_noise_std = 0)
//   composite bwd     autograd of the above
// Arithmetic that decides sample positions or indices uses separately rounded IEEE ops
// (no FMA contraction), like torch's CPU kernels, so indices/positions match bit for bit
// given identical inputs.  Scans over samples run one wave per ray.
#include "common.h"

namespace nerf {

// ------------------------------------------------------------------------------------
// rays
// ------------------------------------------------------------------------------------
struct RaygenArgs {
  const float* c2w;      // [n_img, 4, 4]
  int n_img, H, W;
  float focal;
  const int64_t* pix;    // [R] flat ids img*H*W + j*W + i, or null (then drawn uniformly)
  int64_t R;
  uint64_t seed, offset;
  const float* images;   // [n_img, H, W, 3] or null
  float* rays;           // [R, 6]
  float* rgb;            // [R, 3] or null
  int64_t* pix_out;      // [R] or null
};

__global__ void raygen_kernel(RaygenArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.R) return;
  const int64_t npix = (int64_t)a.H * a.W;
  const int64_t total = npix * a.n_img;
  int64_t id;
  if (a.pix) {
    id = a.pix[r];
  } else {
    // 53-bit draw -> [0, total)
    uint4 c = make_uint4((uint32_t)r, (uint32_t)(r >> 32), (uint32_t)a.offset, (uint32_t)(a.offset >> 32));
    uint4 q = philox(c, make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32)));
    uint64_t x = ((uint64_t)q.x << 21) ^ (uint64_t)q.y;
    id = (int64_t)(((unsigned __int128)x * (unsigned __int128)total) >> 53);
  }
  if (a.pix_out) a.pix_out[r] = id;
  const int img = (int)(id / npix);
  const int64_t p = id - (int64_t)img * npix;
  const int j = (int)(p / a.W), i = (int)(p - (int64_t)j * a.W);
  const float* m = a.c2w + (int64_t)img * 16;
  // dirs = ((i - W/2) / f, -(j - H/2) / f, -1)   (blender.py:22-24)
  const float x = fdiv(fsub((float)i, (float)a.W * 0.5f), a.focal);
  const float y = fdiv(-fsub((float)j, (float)a.H * 0.5f), a.focal);
  const float z = -1.f;
  float* o = a.rays + r * 6;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    o[3 + k] = fadd(fadd(fmul(m[4 * k + 0], x), fmul(m[4 * k + 1], y)), fmul(m[4 * k + 2], z));
    o[k] = m[4 * k + 3];
  }
  if (a.rgb) {
    const float* src = a.images + id * 3;
    a.rgb[r * 3 + 0] = src[0];
    a.rgb[r * 3 + 1] = src[1];
    a.rgb[r * 3 + 2] = src[2];
  }
}

// ------------------------------------------------------------------------------------
// stratified depths + sample points + unit view dirs
// ------------------------------------------------------------------------------------
struct StratArgs {
  const float* rays;  // [R,6]
  int64_t R;
  int S;
  const float* t_lin;  // [S] = torch.linspace(0,1,S) (CPU table)
  const float* near;   // device scalars
  const float* far;
  int perturb;
  const float* t_rand;  // [R,S] or null (then philox)
  uint64_t seed, offset;
  float* z;         // [R,S]
  float* pts;       // [R,S,3] or null
  float* viewdirs;  // [R,3] or null
};

__device__ __forceinline__ float strat_base(const float* t_lin, int s, float nr, float fr) {
  const float t = t_lin[s];
  return fadd(fmul(nr, fsub(1.f, t)), fmul(fr, t));  // near * (1 - t) + far * t
}

__global__ void stratified_kernel(StratArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.R * a.S) return;
  const int64_t r = i / a.S;
  const int s = (int)(i - r * a.S);
  const float nr = *a.near, fr = *a.far;
  float z = strat_base(a.t_lin, s, nr, fr);
  if (a.perturb) {
    const float zl = s > 0 ? strat_base(a.t_lin, s - 1, nr, fr) : z;
    const float zu = s + 1 < a.S ? strat_base(a.t_lin, s + 1, nr, fr) : z;
    const float lower = s > 0 ? fmul(0.5f, fadd(z, zl)) : z;      // .5 * (z[1:] + z[:-1])
    const float upper = s + 1 < a.S ? fmul(0.5f, fadd(zu, z)) : z;
    const float u = a.t_rand ? a.t_rand[i] : rng_uniform(a.seed, a.offset, (uint64_t)i);
    z = fadd(lower, fmul(fsub(upper, lower), u));
  }
  a.z[i] = z;
  const float* ray = a.rays + r * 6;
  if (a.pts) {
#pragma unroll
    for (int k = 0; k < 3; ++k) a.pts[i * 3 + k] = fadd(ray[k], fmul(ray[3 + k], z));
  }
  if (a.viewdirs && s == 0) {
    const float dx = ray[3], dy = ray[4], dz = ray[5];
    const float n = sqrtf(fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz)));
    a.viewdirs[r * 3 + 0] = fdiv(dx, n);
    a.viewdirs[r * 3 + 1] = fdiv(dy, n);
    a.viewdirs[r * 3 + 2] = fdiv(dz, n);
  }
}

// ------------------------------------------------------------------------------------
// wave-level searchsorted(right=True) over a sorted array held one entry per lane
// (lanes >= n hold +inf): returns #entries <= u, in [0, n]
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int wave_searchsorted_right(float cdf_lane, float u) {
  int lo = 0, hi = 64;
#pragma unroll
  for (int it = 0; it < 7; ++it) {
    const int mid = (lo + hi) >> 1;
    const float c = __shfl(cdf_lane, mid < 64 ? mid : 63, 64);
    const bool le = mid < 64 && c <= u;
    if (lo < hi) {
      if (le) lo = mid + 1;
      else hi = mid;
    }
  }
  return lo;
}

struct SearchArgs {
  const float* cdf;  // [R, nb]
  const float* u;    // [R, n]
  int64_t R;
  int nb, n;
  int32_t* inds;     // [R, n]
};

// one wave per row; standalone form of the searchsorted used inside sample_pdf
__global__ void searchsorted_kernel(SearchArgs a) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= a.R) return;
  const int l = lane_id();
  const float c = l < a.nb ? a.cdf[r * a.nb + l] : __builtin_inff();
  for (int i0 = 0; i0 < a.n; i0 += 64) {
    const int i = i0 + l;
    const float u = i < a.n ? a.u[r * a.n + i] : 0.f;
    const int k = wave_searchsorted_right(c, u);
    if (i < a.n) a.inds[r * a.n + i] = k;
  }
}

// ------------------------------------------------------------------------------------
// bitonic sort of 256 values held as 4 registers x 64 lanes (position = 64 k + lane)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void bitonic256(float (&v)[4]) {
  const int l = lane_id();
#pragma unroll
  for (int size = 2; size <= 256; size <<= 1) {
#pragma unroll
    for (int j = size >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int kj = j >> 6;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if ((k & kj) == 0) {
            const int p = 64 * k + l;
            const bool asc = (p & size) == 0;
            const float a = v[k], b = v[k ^ kj];
            const float lo = fminf(a, b), hi = fmaxf(a, b);
            v[k] = asc ? lo : hi;
            v[k ^ kj] = asc ? hi : lo;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int p = 64 * k + l;
          const bool asc = (p & size) == 0;
          const float o = __shfl_xor(v[k], j, 64);
          const bool lower = (l & j) == 0;
          v[k] = (lower == asc) ? fminf(v[k], o) : fmaxf(v[k], o);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// importance sampling + merge with the coarse depths (one wave per ray)
// supports Sc <= 64 coarse samples (Sc-1 CDF entries), Ni <= 128, Sc + Ni <= 256
// ------------------------------------------------------------------------------------
struct PdfArgs {
  const float* z;        // [R, Sc]
  const float* weights;  // [R, Sc] (the coarse weights; entries 1..Sc-2 are used)
  int64_t R;
  int Sc, Ni;
  int det;
  const float* u_lin;    // [Ni] linspace(0,1,Ni) table (det)
  const float* u;        // [R, Ni] or null
  uint64_t seed, offset;
  const float* rays;     // [R,6] or null (for pts)
  float* z_fine;         // [R, Sc+Ni]
  float* pts_fine;       // [R, Sc+Ni, 3] or null
  float* samples;        // [R, Ni] or null (unsorted, in u order)
  float* cdf_out;        // [R, Sc-1] or null
  int32_t* inds_out;     // [R, Ni] or null
  // (round 6) per-ray "fragile" flag or null: 1 when some importance sample's bin, or the den < 1e-5 switch
  // of its interval, could change if every CDF entry c moved by up to rel_tol min(c, 1 - c) + abs_tol
  int32_t* fragile;
  float rel_tol, abs_tol, den_tol, z_tol;
};

// one ray (one wave): zc = z of coarse sample l (l < Sc), wn = its weight of sample l + 1
// (l < Sc - 2) -- from memory (sample_pdf_kernel) or from the compositing registers
// (composite_pdf_kernel), the same fp32 values either way
__device__ __forceinline__ void sample_pdf_ray(const PdfArgs& a, int64_t r, int l, float zc, float wn) {
  const int nb = a.Sc - 1;  // bins (z mids) and CDF entries
  const int nw = a.Sc - 2;  // pdf weights
  const float zn = __shfl(zc, l + 1 < 64 ? l + 1 : 63, 64);
  const float bin = l < nb ? fmul(0.5f, fadd(zn, zc)) : 0.f;  // .5 * (z[1:] + z[:-1])
  const float w = l < nw ? fadd(wn, 1e-5f) : 0.f;
  const float wsum = torch_row_sum(w, nw);  // the CPU torch.sum's order (common.h)
  const float pdf = l < nw ? fdiv(w, wsum) : 0.f;
  // cdf[0] = 0, cdf[k] = fp32(sum_{j<k} pdf_j) accumulated in double (torch CPU cumsum)
  const double incl = wave_scan_add((double)pdf);
  const double excl = __shfl_up(incl, 1, 64);
  float cdf = l == 0 ? 0.f : (float)excl;
  if (l >= nb) cdf = __builtin_inff();
  if (a.cdf_out && l < nb) a.cdf_out[r * nb + l] = cdf;

  float v[4];
  v[0] = l < a.Sc ? zc : __builtin_inff();
  bool frag = false;
  // the last two CDF entries (the u = 1 end case of the fragile flag)
  const float c_last = __shfl(cdf, nb - 1, 64), c_prev = __shfl(cdf, nb > 1 ? nb - 2 : 0, 64);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = l + 64 * q;
    float s = __builtin_inff();
    // all lanes take part in the shuffles of the search
    float u = 0.f;
    if (i < a.Ni) {
      u = a.det ? a.u_lin[i] : (a.u ? a.u[r * a.Ni + i] : rng_uniform(a.seed, a.offset, (uint64_t)(r * a.Ni + i)));
    }
    const int ind = wave_searchsorted_right(cdf, u);
    const int below = ind - 1 > 0 ? ind - 1 : 0;
    const int above = ind < nb - 1 ? ind : nb - 1;
    const float cb = __shfl(cdf, below, 64), ca = __shfl(cdf, above, 64);
    const float bb = __shfl(bin, below, 64), ba = __shfl(bin, above, 64);
    if (i < a.Ni) {
      const float den0 = fsub(ca, cb);
      const float den = den0 < 1e-5f ? 1.f : den0;
      const float t = fdiv(fsub(u, cb), den);
      s = fadd(bb, fmul(t, fsub(ba, bb)));
      if (a.samples) a.samples[r * a.Ni + i] = s;
      if (a.inds_out) a.inds_out[r * a.Ni + i] = ind;
      if (a.fragile) {
        // the bin of u changes iff an entry crosses u: its neighbours cdf[ind - 1] <= u < cdf[ind] (cdf[0] = 0 is
        // exact).  The last entry against u = 1 (the linspace's end) is its own case: with cdf[nb-1] <= 1 the
        // sample is the last bin edge, with cdf[nb-1] > 1 it is that edge too -- unless the last interval's pdf
        // is below the 1e-5 switch, when it drops to the start of that bin.  So that flip is flagged only when
        // the last entry is within abs_tol of 1 and the last interval is below 1e-5 + den_tol.  The den < 1e-5
        // switch (volume_renderer.py:124) elsewhere is flagged within den_tol of 1e-5
        const bool end = u >= 1.f;
        const float tb = fadd(fmul(a.rel_tol, fminf(cb, fsub(1.f, cb))), a.abs_tol);
        const float ta = fadd(fmul(a.rel_tol, fminf(ca, fsub(1.f, ca))), a.abs_tol);
        if (ind - 1 >= 1 && !(end && ind - 1 == nb - 1) && fsub(u, cb) < tb) frag = true;
        if (ind <= nb - 1 && !(end && ind == nb - 1) && fsub(ca, u) <= ta) frag = true;
        if (below != above && fabsf(fsub(den0, 1e-5f)) <= a.den_tol) frag = true;
        if (end && fabsf(fsub(c_last, 1.f)) <= a.abs_tol && fsub(c_last, c_prev) < fadd(1e-5f, a.den_tol)) frag = true;
        // within a bin the sample moves by (dcb + t ddcb) / den of the bin width: flag a move beyond z_tol
        if (a.z_tol > 0.f && den0 >= 1e-5f && fmul(fdiv(fadd(ta, tb), den0), fsub(ba, bb)) > a.z_tol) frag = true;
      }
    }
    v[1 + q] = s;
  }
  if (a.fragile) {
    const bool any = __ballot(frag) != 0;
    if (l == 0) a.fragile[r] = any ? 1 : 0;
  }
  v[3] = __builtin_inff();
  // positions >= Sc + Ni hold +inf; the first Sc+Ni sorted entries are the merged depths
  bitonic256(v);
  const int S = a.Sc + a.Ni;
  const float* ray = a.rays ? a.rays + r * 6 : nullptr;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = 64 * k + l;
    if (p < S) {
      a.z_fine[r * S + p] = v[k];
      if (a.pts_fine) {
#pragma unroll
        for (int d = 0; d < 3; ++d) a.pts_fine[(r * S + p) * 3 + d] = fadd(ray[d], fmul(ray[3 + d], v[k]));
      }
    }
  }
}

__global__ void __launch_bounds__(256) sample_pdf_kernel(PdfArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.R) return;
  const int l = lane_id();
  const float zc = l < a.Sc ? a.z[r * a.Sc + l] : 0.f;
  const float wn = l < a.Sc - 2 ? a.weights[r * a.Sc + l + 1] : 0.f;
  sample_pdf_ray(a, r, l, zc, wn);
}

// reference-signature form: sample_pdf(bins [R,nb], weights [R,nb-1], N, det) -> samples
struct PdfBinsArgs {
  const float* bins;
  const float* weights;
  int64_t R;
  int nb, Ni, det;
  const float* u_lin;
  const float* u;
  uint64_t seed, offset;
  float* samples;   // [R, Ni]
  float* cdf_out;   // [R, nb] or null
  int32_t* inds_out;
};

__global__ void __launch_bounds__(256) sample_pdf_bins_kernel(PdfBinsArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.R) return;
  const int l = lane_id();
  const int nw = a.nb - 1;
  const float bin = l < a.nb ? a.bins[r * a.nb + l] : 0.f;
  const float w = l < nw ? fadd(a.weights[r * nw + l], 1e-5f) : 0.f;
  const float wsum = torch_row_sum(w, nw);
  const float pdf = l < nw ? fdiv(w, wsum) : 0.f;
  const double incl = wave_scan_add((double)pdf);
  const double excl = __shfl_up(incl, 1, 64);
  float cdf = l == 0 ? 0.f : (float)excl;
  if (l >= a.nb) cdf = __builtin_inff();
  if (a.cdf_out && l < a.nb) a.cdf_out[r * a.nb + l] = cdf;
  for (int i0 = 0; i0 < a.Ni; i0 += 64) {
    const int i = i0 + l;
    float u = 0.f;
    if (i < a.Ni) u = a.det ? a.u_lin[i] : (a.u ? a.u[r * a.Ni + i] : rng_uniform(a.seed, a.offset, (uint64_t)(r * a.Ni + i)));
    const int ind = wave_searchsorted_right(cdf, u);
    const int below = ind - 1 > 0 ? ind - 1 : 0;
    const int above = ind < a.nb - 1 ? ind : a.nb - 1;
    const float cb = __shfl(cdf, below, 64), ca = __shfl(cdf, above, 64);
    const float bb = __shfl(bin, below, 64), ba = __shfl(bin, above, 64);
    if (i < a.Ni) {
      float den = fsub(ca, cb);
      den = den < 1e-5f ? 1.f : den;
      const float t = fdiv(fsub(u, cb), den);
      a.samples[r * a.Ni + i] = fadd(bb, fmul(t, fsub(ba, bb)));
      if (a.inds_out) a.inds_out[r * a.Ni + i] = ind;
    }
  }
}

// ------------------------------------------------------------------------------------
// alpha compositing, one wave per ray, SPL = samples per lane (S <= 64 SPL)
// ------------------------------------------------------------------------------------
struct CompArgs {
  const float* raw;   // [R,S,4]
  const float* z;     // [R,S]
  const float* dirs;  // [R, dir_stride] (d in the first 3)
  int dir_stride;
  int64_t R;
  int S;
  int white;
  // forward outputs
  float* rgb;      // [R,3]
  float* depth;    // [R]
  float* acc;      // [R]
  float* weights;  // [R,S] or null
  // backward
  const float* g_rgb;    // [R,3]
  const float* g_depth;  // [R] or null
  const float* g_acc;    // [R] or null
  float* g_raw;          // [R,S,4]
};

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

template <int SPL, bool BWD>
__device__ __forceinline__ void composite_ray(const CompArgs& a, int64_t r, int l, float (&w_out)[SPL],
                                              float (&z_out)[SPL]) {
  const int S = a.S;
  const float dx = a.dirs[r * a.dir_stride + 0], dy = a.dirs[r * a.dir_stride + 1],
              dz = a.dirs[r * a.dir_stride + 2];
  const float dn = sqrtf(fadd(fadd(fmul(dx, dx), fmul(dy, dy)), fmul(dz, dz)));
  float zs[SPL], alpha[SPL], x[SPL], sig[SPL], delta[SPL], c[SPL][3];
  bool pos[SPL];
  const int s0 = l * SPL;
  // the depth after this lane's last sample (for the last delta)
  const float z_after_local = (s0 + SPL < S) ? a.z[r * S + s0 + SPL] : 0.f;
#pragma unroll
  for (int k = 0; k < SPL; ++k) {
    const int s = s0 + k;
    const bool ok = s < S;
    zs[k] = ok ? a.z[r * S + s] : 0.f;
    float4 rw = ok ? *(const float4*)(a.raw + (r * S + s) * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
    c[k][0] = sigmoidf_(rw.x);
    c[k][1] = sigmoidf_(rw.y);
    c[k][2] = sigmoidf_(rw.z);
    pos[k] = rw.w > 0.f;
    sig[k] = pos[k] ? rw.w : 0.f;
  }
#pragma unroll
  for (int k = 0; k < SPL; ++k) {
    const int s = s0 + k;
    float zn = (k + 1 < SPL) ? zs[k + 1] : z_after_local;
    float d = s + 1 < S ? fsub(zn, zs[k]) : 1e10f;
    d = fmul(d, dn);
    delta[k] = d;
    alpha[k] = s < S ? fsub(1.f, expf(-fmul(sig[k], d))) : 0.f;
    x[k] = s < S ? fadd(fsub(1.f, alpha[k]), 1e-10f) : 1.f;
  }
  // exclusive product scan in double
  double lp = 1.0;
#pragma unroll
  for (int k = 0; k < SPL; ++k) lp *= (double)x[k];
  const double incl = wave_scan_mul(lp);
  double run = __shfl_up(incl, 1, 64);
  if (l == 0) run = 1.0;
  float T[SPL], w[SPL];
#pragma unroll
  for (int k = 0; k < SPL; ++k) {
    T[k] = (float)run;
    run *= (double)x[k];
    w[k] = fmul(alpha[k], T[k]);
    w_out[k] = w[k];
    z_out[k] = zs[k];
  }
  if (!BWD) {
    float sr = 0.f, sg = 0.f, sb = 0.f, sd = 0.f, sa = 0.f;
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      sr += w[k] * c[k][0];
      sg += w[k] * c[k][1];
      sb += w[k] * c[k][2];
      sd += w[k] * zs[k];
      sa += w[k];
      if (a.weights && s0 + k < S) a.weights[r * S + s0 + k] = w[k];
    }
    sr = wave_sum(sr);
    sg = wave_sum(sg);
    sb = wave_sum(sb);
    sd = wave_sum(sd);
    sa = wave_sum(sa);
    if (l == 0) {
      if (a.white) {
        const float bg = fsub(1.f, sa);
        sr = fadd(sr, bg);
        sg = fadd(sg, bg);
        sb = fadd(sb, bg);
      }
      a.rgb[r * 3 + 0] = sr;
      a.rgb[r * 3 + 1] = sg;
      a.rgb[r * 3 + 2] = sb;
      a.depth[r] = sd;
      a.acc[r] = sa;
    }
  } else {
    const float g0 = a.g_rgb[r * 3 + 0], g1 = a.g_rgb[r * 3 + 1], g2 = a.g_rgb[r * 3 + 2];
    const float gd = a.g_depth ? a.g_depth[r] : 0.f;
    float ga = a.g_acc ? a.g_acc[r] : 0.f;
    if (a.white) ga -= (g0 + g1) + g2;  // rgb += 1 - acc
    float e[SPL], ew_local = 0.f;
#pragma unroll
    for (int k = 0; k < SPL; ++k) {
      e[k] = g0 * c[k][0] + g1 * c[k][1] + g2 * c[k][2] + gd * zs[k] + ga;  // dL/dw
      ew_local += e[k] * w[k];
    }
    // suffix sums of e*w: total - inclusive prefix
    const float incl_ew = wave_scan_add_f(ew_local);
    const float total = __shfl(incl_ew, 63, 64);
    float after = total - incl_ew;  // sum over later lanes
#pragma unroll
    for (int k = SPL - 1; k >= 0; --k) {
      const int s = s0 + k;
      // dL/dalpha_k = e_k T_k - (sum_{i>k} e_i w_i) / x_k
      const float dA = e[k] * T[k] - after / x[k];
      after += e[k] * w[k];
      const float dsig = dA * delta[k] * expf(-sig[k] * delta[k]);
      const float d3 = pos[k] ? dsig : 0.f;
      const float wr = w[k];
      if (s < S) {
        float4 o = make_float4(wr * g0 * c[k][0] * (1.f - c[k][0]), wr * g1 * c[k][1] * (1.f - c[k][1]),
                               wr * g2 * c[k][2] * (1.f - c[k][2]), d3);
        *(float4*)(a.g_raw + (r * S + s) * 4) = o;
      }
    }
  }
}

template <int SPL, bool BWD>
__global__ void __launch_bounds__(256) composite_kernel(CompArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.R) return;
  float w[SPL], z[SPL];
  composite_ray<SPL, BWD>(a, r, lane_id(), w, z);
}

// the coarse pass's compositing and the importance sampling + merge that reads its weights,
// fused (volume_renderer.py:197-221): one wave per ray, the weights handed over in registers
__global__ void __launch_bounds__(256) composite_pdf_kernel(CompArgs c, PdfArgs p) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= c.R) return;
  const int l = lane_id();
  float w[1], z[1];
  composite_ray<1, false>(c, r, l, w, z);
  const float wn = __shfl(w[0], l + 1 < 64 ? l + 1 : 63, 64);  // weight of sample l + 1
  sample_pdf_ray(p, r, l, l < c.S ? z[0] : 0.f, l < c.S - 2 ? wn : 0.f);
}

}  // namespace nerf

// ======================================================================================
// C-ABI
// ======================================================================================
using namespace nerf;

extern "C" {

int nerf_raygen(const float* c2w, int n_img, int H, int W, float focal, const int64_t* pix, int64_t R,
                uint64_t seed, uint64_t offset, const float* images, float* rays, float* rgb, int64_t* pix_out,
                hipStream_t stream) {
  NERF_REQUIRE(R >= 0 && n_img > 0 && H > 0 && W > 0, "nerf_raygen: bad sizes");
  if (R == 0) return 0;
  NERF_REQUIRE(c2w && rays, "nerf_raygen: null pointer");
  NERF_REQUIRE(!rgb || images, "nerf_raygen: rgb output needs images");
  RaygenArgs a{c2w, n_img, H, W, focal, pix, R, seed, offset, images, rays, rgb, pix_out};
  hipLaunchKernelGGL(raygen_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, stream, a);
  return check_launch("nerf_raygen");
}

int nerf_sample_stratified(const float* rays, int64_t R, int S, const float* t_lin, const float* near,
                           const float* far, int perturb, const float* t_rand, uint64_t seed, uint64_t offset,
                           float* z, float* pts, float* viewdirs, hipStream_t stream) {
  NERF_REQUIRE(R >= 0 && S > 0, "nerf_sample_stratified: bad sizes");
  if (R == 0) return 0;
  NERF_REQUIRE(rays && t_lin && near && far && z, "nerf_sample_stratified: null pointer");
  StratArgs a{rays, R, S, t_lin, near, far, perturb, t_rand, seed, offset, z, pts, viewdirs};
  hipLaunchKernelGGL(stratified_kernel, dim3((unsigned)((R * S + 255) / 256)), dim3(256), 0, stream, a);
  return check_launch("nerf_sample_stratified");
}

int nerf_searchsorted(const float* cdf, const float* u, int64_t R, int nb, int n, int32_t* inds,
                      hipStream_t stream) {
  NERF_REQUIRE(nb > 0 && nb <= 64 && n >= 0 && R >= 0, "nerf_searchsorted: need 0 < nb <= 64");
  if (R == 0 || n == 0) return 0;
  NERF_REQUIRE(cdf && u && inds, "nerf_searchsorted: null pointer");
  SearchArgs a{cdf, u, R, nb, n, inds};
  hipLaunchKernelGGL(searchsorted_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, a);
  return check_launch("nerf_searchsorted");
}

int nerf_sample_pdf(const float* z, const float* weights, int64_t R, int Sc, int Ni, int det, const float* u_lin,
                    const float* u, uint64_t seed, uint64_t offset, const float* rays, float* z_fine,
                    float* pts_fine, float* samples, float* cdf_out, int32_t* inds_out, hipStream_t stream) {
  NERF_REQUIRE(Sc >= 3 && Sc <= 64 && Ni >= 1 && Ni <= 128 && Sc + Ni <= 256,
               "nerf_sample_pdf: need 3 <= Sc <= 64, 1 <= Ni <= 128 (got %d, %d)", Sc, Ni);
  NERF_REQUIRE(R >= 0, "nerf_sample_pdf: R < 0");
  if (R == 0) return 0;
  NERF_REQUIRE(z && weights && z_fine, "nerf_sample_pdf: null pointer");
  NERF_REQUIRE(!det || u_lin, "nerf_sample_pdf: det needs the linspace table");
  NERF_REQUIRE(!pts_fine || rays, "nerf_sample_pdf: pts_fine needs rays");
  PdfArgs a{z, weights, R, Sc, Ni, det, u_lin, u, seed, offset, rays, z_fine, pts_fine, samples, cdf_out, inds_out};
  hipLaunchKernelGGL(sample_pdf_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, a);
  return check_launch("nerf_sample_pdf");
}

int nerf_sample_pdf_bins(const float* bins, const float* weights, int64_t R, int nb, int Ni, int det,
                         const float* u_lin, const float* u, uint64_t seed, uint64_t offset, float* samples,
                         float* cdf_out, int32_t* inds_out, hipStream_t stream) {
  NERF_REQUIRE(nb >= 2 && nb <= 64 && Ni >= 1 && R >= 0, "nerf_sample_pdf_bins: need 2 <= nb <= 64, Ni >= 1");
  if (R == 0) return 0;
  NERF_REQUIRE(bins && weights && samples, "nerf_sample_pdf_bins: null pointer");
  NERF_REQUIRE(!det || u_lin, "nerf_sample_pdf_bins: det needs the linspace table");
  PdfBinsArgs a{bins, weights, R, nb, Ni, det, u_lin, u, seed, offset, samples, cdf_out, inds_out};
  hipLaunchKernelGGL(sample_pdf_bins_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, a);
  return check_launch("nerf_sample_pdf_bins");
}

static int composite_launch(CompArgs& a, bool bwd, hipStream_t stream) {
  const int spl = (a.S + 63) / 64;
  dim3 grid((unsigned)((a.R + 3) / 4)), block(256);
#define NERF_COMP(N)                                                                          \
  if (spl == N) {                                                                             \
    if (bwd) hipLaunchKernelGGL((composite_kernel<N, true>), grid, block, 0, stream, a);      \
    else hipLaunchKernelGGL((composite_kernel<N, false>), grid, block, 0, stream, a);         \
  }
  NERF_COMP(1) NERF_COMP(2) NERF_COMP(3) NERF_COMP(4)
#undef NERF_COMP
  return check_launch(bwd ? "nerf_composite_bwd" : "nerf_composite_fwd");
}

int nerf_composite_fwd(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int S,
                       int white_bkgd, float* rgb, float* depth, float* acc, float* weights, hipStream_t stream) {
  NERF_REQUIRE(S >= 1 && S <= 256 && R >= 0 && dir_stride >= 3, "nerf_composite_fwd: need 1 <= S <= 256");
  if (R == 0) return 0;
  NERF_REQUIRE(raw && z && dirs && rgb && depth && acc, "nerf_composite_fwd: null pointer");
  CompArgs a{raw, z, dirs, dir_stride, R, S, white_bkgd, rgb, depth, acc, weights, nullptr, nullptr, nullptr, nullptr};
  return composite_launch(a, false, stream);
}

int nerf_composite_pdf(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int Sc,
                       int white_bkgd, float* rgb, float* depth, float* acc, float* weights, int Ni, int det,
                       const float* u_lin, const float* u, uint64_t seed, uint64_t offset, const float* rays,
                       float* z_fine, float* pts_fine, hipStream_t stream) {
  NERF_REQUIRE(Sc >= 3 && Sc <= 64 && Ni >= 1 && Ni <= 128 && Sc + Ni <= 256 && R >= 0 && dir_stride >= 3,
               "nerf_composite_pdf: need 3 <= Sc <= 64, 1 <= Ni <= 128 (got %d, %d)", Sc, Ni);
  if (R == 0) return 0;
  NERF_REQUIRE(raw && z && dirs && rgb && depth && acc && z_fine, "nerf_composite_pdf: null pointer");
  NERF_REQUIRE(!det || u_lin, "nerf_composite_pdf: det needs the linspace table");
  NERF_REQUIRE(!pts_fine || rays, "nerf_composite_pdf: pts_fine needs rays");
  CompArgs c{raw, z, dirs, dir_stride, R, Sc, white_bkgd, rgb, depth, acc, weights, nullptr, nullptr, nullptr, nullptr};
  PdfArgs p{z, nullptr, R, Sc, Ni, det, u_lin, u, seed, offset, rays, z_fine, pts_fine, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(composite_pdf_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, c, p);
  return check_launch("nerf_composite_pdf");
}

int nerf_composite_pdf_fragile(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int Sc,
                               int white_bkgd, float* rgb, float* depth, float* acc, int Ni, const float* u_lin,
                               const float* rays, float* z_fine, float* pts_fine, float rel_tol, float abs_tol,
                               float den_tol, float z_tol, int32_t* fragile, hipStream_t stream) {
  NERF_REQUIRE(Sc >= 3 && Sc <= 64 && Ni >= 1 && Ni <= 128 && Sc + Ni <= 256 && R >= 0 && dir_stride >= 3,
               "nerf_composite_pdf_fragile: need 3 <= Sc <= 64, 1 <= Ni <= 128 (got %d, %d)", Sc, Ni);
  if (R == 0) return 0;
  NERF_REQUIRE(raw && z && dirs && rgb && depth && acc && z_fine && u_lin && fragile,
               "nerf_composite_pdf_fragile: null pointer");
  NERF_REQUIRE(!pts_fine || rays, "nerf_composite_pdf_fragile: pts_fine needs rays");
  NERF_REQUIRE(rel_tol >= 0.f && abs_tol >= 0.f && den_tol >= 0.f && z_tol >= 0.f,
               "nerf_composite_pdf_fragile: negative tolerance");
  CompArgs c{raw, z, dirs, dir_stride, R, Sc, white_bkgd, rgb, depth, acc, nullptr, nullptr, nullptr, nullptr, nullptr};
  PdfArgs p{z, nullptr, R, Sc, Ni, 1, u_lin, nullptr, 0, 0, rays, z_fine, pts_fine, nullptr, nullptr, nullptr,
            fragile, rel_tol, abs_tol, den_tol, z_tol};
  hipLaunchKernelGGL(composite_pdf_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, c, p);
  return check_launch("nerf_composite_pdf_fragile");
}

int nerf_composite_bwd(const float* raw, const float* z, const float* dirs, int dir_stride, int64_t R, int S,
                       int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc, float* g_raw,
                       hipStream_t stream) {
  NERF_REQUIRE(S >= 1 && S <= 256 && R >= 0 && dir_stride >= 3, "nerf_composite_bwd: need 1 <= S <= 256");
  if (R == 0) return 0;
  NERF_REQUIRE(raw && z && dirs && g_rgb && g_raw, "nerf_composite_bwd: null pointer");
  CompArgs a{raw, z, dirs, dir_stride, R, S, white_bkgd, nullptr, nullptr, nullptr, nullptr, g_rgb, g_depth, g_acc, g_raw};
  return composite_launch(a, true, stream);
}

}  // extern "C"
