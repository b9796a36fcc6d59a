// Image metrics of the evaluator on the GPU: PSNR and scikit-image-style SSIM.
//
// Reference: src/evaluators/nerf.py:23-45 -- psnr = -10 log10(mean((pred - gt)^2)) on the
// float images; ssim = skimage.metrics.structural_similarity(uint8(pred * 255),
// uint8(gt * 255), channel_axis=-1, data_range=pred_u8.max() - pred_u8.min()) with
// skimage's defaults (7x7 uniform window, K1 = 0.01, K2 = 0.03, sample covariance
// N / (N - 1), 3-pixel border cropped before the mean, mean over channels).  The cropped
// pixels' windows lie entirely inside the image, so the filter's border mode never enters.
//
// Window sums of uint8 values, their squares and products are exact integers (<= 49 * 255^2);
// the SSIM formula is evaluated in fp64 like numpy's float64 path.
#include "common.h"

namespace nerf {

struct MetricsWs {
  int pmin, pmax;               // uint8 range of pred
  double sse;                   // sum of squared fp32 differences
  double ssim_sum;              // sum of per-pixel SSIM over the cropped region, all channels
};

__global__ void metrics_u8_kernel(const float* pred, const float* gt, int64_t n, uint8_t* pu8, uint8_t* gu8,
                                  MetricsWs* ws) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double se = 0.0;
  int lo = 255, hi = 0;
  if (i < n) {
    const float p = pred[i], g = gt[i];
    const float d = p - g;
    se = (double)(d * d);  // (pred - gt) ** 2 in float32, as numpy on float32 arrays
    // numpy float32 -> uint8 truncates toward zero (values are in [0, 255] here)
    const int pu = (int)(p * 255.f), gu = (int)(g * 255.f);
    pu8[i] = (uint8_t)pu;
    gu8[i] = (uint8_t)gu;
    lo = hi = pu & 255;
  }
  // wave reductions, one atomic per wave
  for (int o = 32; o > 0; o >>= 1) {
    se += __shfl_xor(se, o, 64);
    lo = min(lo, __shfl_xor(lo, o, 64));
    hi = max(hi, __shfl_xor(hi, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&ws->sse, se);
    atomicMin(&ws->pmin, lo);
    atomicMax(&ws->pmax, hi);
  }
}

// one thread per (cropped pixel, channel)
__global__ void ssim_kernel(const uint8_t* pu8, const uint8_t* gu8, int H, int W, MetricsWs* ws) {
  const int Hc = H - 6, Wc = W - 6;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double s = 0.0;
  if (t < (int64_t)Hc * Wc * 3) {
    const int c = (int)(t % 3);
    const int64_t q = t / 3;
    const int y = (int)(q / Wc) + 3, x = (int)(q % Wc) + 3;
    int sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
    for (int dy = -3; dy <= 3; ++dy) {
      const int64_t row = ((int64_t)(y + dy) * W) * 3 + c;
#pragma unroll
      for (int dx = -3; dx <= 3; ++dx) {
        const int a = pu8[row + (int64_t)(x + dx) * 3], b = gu8[row + (int64_t)(x + dx) * 3];
        sx += a;
        sy += b;
        sxx += a * a;
        syy += b * b;
        sxy += a * b;
      }
    }
    const double N = 49.0, cov = N / (N - 1.0);
    const double ux = sx / N, uy = sy / N;
    const double vx = cov * (sxx / N - ux * ux), vy = cov * (syy / N - uy * uy), vxy = cov * (sxy / N - ux * uy);
    const double dr = (double)(ws->pmax - ws->pmin);
    const double C1 = (0.01 * dr) * (0.01 * dr), C2 = (0.03 * dr) * (0.03 * dr);
    s = ((2.0 * ux * uy + C1) * (2.0 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2));
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(&ws->ssim_sum, s);
}

__global__ void metrics_init_kernel(MetricsWs* ws) {
  ws->pmin = 255;
  ws->pmax = 0;
  ws->sse = 0.0;
  ws->ssim_sum = 0.0;
}

__global__ void metrics_finish_kernel(const MetricsWs* ws, int64_t n, int64_t ncrop, double* out) {
  out[0] = -10.0 * log10(ws->sse / (double)n);
  out[1] = ws->ssim_sum / (double)ncrop;
  out[2] = ws->sse;
  out[3] = (double)(ws->pmax - ws->pmin);
}

}  // namespace nerf

using namespace nerf;

extern "C" {

int64_t nerf_metrics_workspace_bytes(int H, int W) {
  if (H <= 0 || W <= 0) return -1;
  return 256 + 2 * (int64_t)H * W * 3;
}

int nerf_image_metrics(const float* pred, const float* gt, int H, int W, void* workspace, double* out,
                       hipStream_t stream) {
  NERF_REQUIRE(pred && gt && workspace && out, "nerf_image_metrics: null pointer");
  NERF_REQUIRE(H > 6 && W > 6, "nerf_image_metrics: image must be larger than the 7x7 SSIM window (%d x %d)", H, W);
  MetricsWs* ws = (MetricsWs*)workspace;
  uint8_t* pu8 = (uint8_t*)workspace + 256;
  uint8_t* gu8 = pu8 + (int64_t)H * W * 3;
  const int64_t n = (int64_t)H * W * 3, ncrop = (int64_t)(H - 6) * (W - 6) * 3;
  hipLaunchKernelGGL(metrics_init_kernel, dim3(1), dim3(1), 0, stream, ws);
  hipLaunchKernelGGL(metrics_u8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, pred, gt, n, pu8, gu8,
                     ws);
  hipLaunchKernelGGL(ssim_kernel, dim3((unsigned)((ncrop + 255) / 256)), dim3(256), 0, stream, pu8, gu8, H, W, ws);
  hipLaunchKernelGGL(metrics_finish_kernel, dim3(1), dim3(1), 0, stream, ws, n, ncrop, out);
  return check_launch("nerf_image_metrics");
}

}  // extern "C"
