// Fused Adam / AMSGrad over one flat parameter buffer (torch.optim.Adam semantics, the
// optimiser of latice/lightning_module.py:26-28 and conf/lightning_module/default.yaml:10-13).
// Replaces ~7 elementwise passes of the foreach implementation by one read of
// {p, g, m, v[, vmax]} and one write of {p, m, v[, vmax]}.  The step counter lives on the
// device (incremented by a 1-thread kernel in front), so the update is graph-capturable.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

__global__ void adam_tick_kernel(float* step) { *step += 1.f; }

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   float* __restrict__ vmax,
                                                   const float* __restrict__ step, int64_t n, float lr,
                                                   float b1, float b2, float eps, float wd) {
  const float t = *step;
  const float bc1 = 1.f - powf(b1, t);
  const float bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i];
    const float pi = p[i];
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);      // exp_avg.lerp_(grad, 1 - beta1)
    const float vi = fmaf(b2, v[i], (1.f - b2) * gi * gi);  // mul_(beta2).addcmul_(g, g, 1-beta2)
    m[i] = mi;
    v[i] = vi;
    float vv = vi;
    if (vmax) {
      vv = fmaxf(vmax[i], vi);
      vmax[i] = vv;
    }
    const float denom = sqrtf(vv) / bc2s + eps;
    p[i] = pi - step_size * (mi / denom);
  }
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_adam(float* p, const float* g, float* m, float* v, float* vmax, float* step,
                            int64_t n, float lr, float beta1, float beta2, float eps,
                            float weight_decay, int amsgrad, ebsdvae_stream_t stream) {
  EV_REQUIRE(p && g && m && v && step && n > 0, "adam: null pointer");
  EV_REQUIRE(!amsgrad || vmax, "adam: amsgrad needs vmax");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(1), 0, s, step);
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v,
                     amsgrad ? vmax : nullptr, step, n, lr, beta1, beta2, eps, weight_decay);
  return evh::check_launch("adam");
}
