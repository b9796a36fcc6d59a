// Fused clip_grad_value_ + Adam step over flat parameter / gradient / moment buffers.
//
// Reference: src/train/trainers/trainer.py:61-62 (torch.nn.utils.clip_grad_value_(40),
// optimizer.step()) with src/train/optimizer.py:8-28 (torch.optim.Adam, one param group
// per tensor, lr 5e-4, betas (0.9, 0.999), eps 1e-8, weight_decay 0).  The reference runs
// ~48 x 10 small ATen kernels per step; here one launch updates all 1,191,688 values.
#include "common.h"

namespace nerf {

struct AdamArgs {
  float* p;
  float* g;
  float* m;
  float* v;
  int64_t n;
  float lr_over_bc1;     // lr / (1 - beta1^t)
  float inv_bc2_sqrt;    // 1 / sqrt(1 - beta2^t)  (used as division by sqrt(bc2))
  float bc2_sqrt;
  float beta1, beta2, eps, clip;
};

__global__ void adam_kernel(AdamArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  float g = a.g[i];
  if (a.clip > 0.f) {
    g = fminf(fmaxf(g, -a.clip), a.clip);
    a.g[i] = g;
  }
  float m = a.m[i], v = a.v[i];
  m = fadd(m, fmul(1.f - a.beta1, fsub(g, m)));        // exp_avg.lerp_(grad, 1 - beta1)
  v = fadd(fmul(v, a.beta2), fmul(1.f - a.beta2, fmul(g, g)));  // mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = fadd(fdiv(sqrtf(v), a.bc2_sqrt), a.eps);
  a.p[i] = fadd(a.p[i], fmul(-a.lr_over_bc1, fdiv(m, denom)));
  a.m[i] = m;
  a.v[i] = v;
}

}  // namespace nerf

using namespace nerf;

extern "C" {

// step = the Adam step count after increment (1 for the first update)
int nerf_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr, double beta1,
                   double beta2, double eps, int64_t step, double clip_value, hipStream_t stream) {
  NERF_REQUIRE(n >= 0 && step >= 1, "nerf_adam_step: bad arguments");
  if (n == 0) return 0;
  NERF_REQUIRE(param && grad && exp_avg && exp_avg_sq, "nerf_adam_step: null pointer");
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  AdamArgs a{param, grad, exp_avg, exp_avg_sq, n, (float)(lr / bc1), (float)(1.0 / std::sqrt(bc2)),
             (float)std::sqrt(bc2), (float)beta1, (float)beta2, (float)eps, (float)clip_value};
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return check_launch("nerf_adam_step");
}

}  // extern "C"
