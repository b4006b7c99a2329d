// VAE loss of latice/lightning_module.py:79-156, forward and backward.
//   recon_b = mean_{c,h,w} BCEWithLogits(x_hat, x)      (:79-92, reduction none + mean(1,2,3))
//   kl_b    = kl_lambda * mean_j [log N(z; mu, std) - log N(z; 0, 1)]
//           = kl_lambda * mean_j [0.5 z^2 - 0.5 ((z - mu)/std)^2 - log std]   (:94-120)
//   elbo_b  = kl_b + recon_b ; loss = mean elbo ; kl_loss = mean kl ; recon_loss = mean recon
// One workgroup per pattern for the per-sample reductions (wave64 shuffles, then 4-wave
// LDS combine, fixed order), one single-workgroup pass for the batch means.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

EV_DEVINL float bce_logits(float x, float y) {
  // (1 - y) * x + softplus(-x), softplus(-x) = max(-x, 0) + log1p(exp(-|x|))
  return (1.f - y) * x + fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x)));
}

EV_DEVINL float sigmoidf_(float x) {
  if (x >= 0.f) return 1.f / (1.f + expf(-x));
  const float e = expf(x);
  return e / (1.f + e);
}

__global__ __launch_bounds__(256) void loss_fwd_kernel(
    const float* __restrict__ xh, const float* __restrict__ x, const float* __restrict__ z,
    const float* __restrict__ mu, const float* __restrict__ sd, float lam,
    float* __restrict__ elbo, float* __restrict__ kl, float* __restrict__ recon, int P, int L) {
  __shared__ float red[8];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* xb = xh + (size_t)b * P;
  const float* yb = x + (size_t)b * P;
  float s = 0.f;
  if ((P & 3) == 0) {
    for (int i = tid * 4; i < P; i += 1024) {
      const float4 a = ld4(xb + i), t = ld4(yb + i);
      s += bce_logits(a.x, t.x) + bce_logits(a.y, t.y) + bce_logits(a.z, t.z) + bce_logits(a.w, t.w);
    }
  } else {
    for (int i = tid; i < P; i += 256) s += bce_logits(xb[i], yb[i]);
  }
  float k = 0.f;
  for (int j = tid; j < L; j += 256) {
    const size_t bj = (size_t)b * L + j;
    const float zz = z[bj], m = mu[bj], sdv = sd[bj];
    const float d = (zz - m) / sdv;
    k += 0.5f * zz * zz - 0.5f * d * d - logf(sdv);
  }
  s = wave_sum(s);
  k = wave_sum(k);
  if (lane == 0) { red[wave] = s; red[4 + wave] = k; }
  __syncthreads();
  if (tid == 0) {
    const float rs = (red[0] + red[1] + red[2] + red[3]) / (float)P;
    const float ks = lam * ((red[4] + red[5] + red[6] + red[7]) / (float)L);
    recon[b] = rs;
    kl[b] = ks;
    elbo[b] = ks + rs;
  }
}

// As loss_fwd_kernel with the BCE sums already reduced per row band by ebsdvae_net_end:
// recon_b = sum_t bce_part[b][t] / P (fixed order).
__global__ __launch_bounds__(64) void loss_fwd_parts_kernel(
    const float* __restrict__ bce_part, int T, const float* __restrict__ z,
    const float* __restrict__ mu, const float* __restrict__ sd, float lam,
    float* __restrict__ elbo, float* __restrict__ kl, float* __restrict__ recon, int P, int L) {
  const int b = blockIdx.x, tid = threadIdx.x;
  float k = 0.f;
  for (int j = tid; j < L; j += 64) {
    const size_t bj = (size_t)b * L + j;
    const float zz = z[bj], m = mu[bj], sdv = sd[bj];
    const float d = (zz - m) / sdv;
    k += 0.5f * zz * zz - 0.5f * d * d - logf(sdv);
  }
  k = wave_sum(k);
  if (tid == 0) {
    float r = 0.f;
    for (int t = 0; t < T; ++t) r += bce_part[(size_t)b * T + t];
    const float rs = r / (float)P;
    const float ks = lam * (k / (float)L);
    recon[b] = rs;
    kl[b] = ks;
    elbo[b] = ks + rs;
  }
}

__global__ __launch_bounds__(256) void loss_mean_kernel(const float* __restrict__ elbo,
                                                        const float* __restrict__ kl,
                                                        const float* __restrict__ recon,
                                                        float* __restrict__ o_loss,
                                                        float* __restrict__ o_kl,
                                                        float* __restrict__ o_rec, int B) {
  __shared__ float red[12];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float a = 0.f, k = 0.f, r = 0.f;
  for (int b = tid; b < B; b += 256) { a += elbo[b]; k += kl[b]; r += recon[b]; }
  a = wave_sum(a); k = wave_sum(k); r = wave_sum(r);
  if (lane == 0) { red[wave] = a; red[4 + wave] = k; red[8 + wave] = r; }
  __syncthreads();
  if (tid == 0) {
    const float inv = 1.f / (float)B;
    *o_loss = (red[0] + red[1] + red[2] + red[3]) * inv;
    *o_kl = (red[4] + red[5] + red[6] + red[7]) * inv;
    *o_rec = (red[8] + red[9] + red[10] + red[11]) * inv;
  }
}

__global__ __launch_bounds__(256) void loss_bwd_kernel(
    const float* __restrict__ xh, const float* __restrict__ x, const float* __restrict__ z,
    const float* __restrict__ mu, const float* __restrict__ sd, float lam,
    const float* __restrict__ gl, const float* __restrict__ gk_, const float* __restrict__ gr_,
    const float* __restrict__ gelbo, float scale, float* __restrict__ gxh,
    float* __restrict__ gz, float* __restrict__ gmu, float* __restrict__ gsd,
    float* __restrict__ gx, int B, int P, int L) {
  const int b = blockIdx.y;
  const float invB = 1.f / (float)B;
  const float ge = gelbo ? gelbo[b] : 0.f;
  const float g_loss = gl ? *gl : 0.f, g_kl = gk_ ? *gk_ : 0.f, g_rec = gr_ ? *gr_ : 0.f;
  const float gr = scale * ((g_loss + g_rec) * invB + ge);   // d / d recon_b
  const float gk = scale * ((g_loss + g_kl) * invB + ge);    // d / d kl_b
  const float cr = gr / (float)P;
  const int i0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const float* xb = xh + (size_t)b * P;
  const float* yb = x + (size_t)b * P;
  if (gxh && i0 < P) {   // gxh NULL: the logit gradient comes from ebsdvae_net_end
    if (i0 + 4 <= P && (P & 3) == 0) {
      const float4 a = ld4(xb + i0), t = ld4(yb + i0);
      st4(gxh + (size_t)b * P + i0,
          make_float4(cr * (sigmoidf_(a.x) - t.x), cr * (sigmoidf_(a.y) - t.y),
                      cr * (sigmoidf_(a.z) - t.z), cr * (sigmoidf_(a.w) - t.w)));
      if (gx) st4(gx + (size_t)b * P + i0, make_float4(-cr * a.x, -cr * a.y, -cr * a.z, -cr * a.w));
    } else {
      for (int i = i0; i < P && i < i0 + 4; ++i) {
        gxh[(size_t)b * P + i] = cr * (sigmoidf_(xb[i]) - yb[i]);
        if (gx) gx[(size_t)b * P + i] = -cr * xb[i];
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < L) {
    const int j = threadIdx.x;
    const size_t bj = (size_t)b * L + j;
    const float ck = gk * lam / (float)L;
    const float zz = z[bj], m = mu[bj], s = sd[bj];
    const float d = (zz - m) / (s * s);
    gz[bj] = ck * (zz - d);
    gmu[bj] = ck * d;
    gsd[bj] = ck * ((zz - m) * (zz - m) / (s * s * s) - 1.f / s);
  }
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_vae_loss_fwd(const float* x_hat, const float* x, const float* z,
                                    const float* mu, const float* std, float kl_lambda,
                                    float* elbo, float* kl, float* recon, float* loss,
                                    float* kl_loss, float* recon_loss, int B, int P, int L,
                                    ebsdvae_stream_t stream) {
  EV_REQUIRE(x_hat && x && z && mu && std && elbo && kl && recon && loss && kl_loss && recon_loss,
             "vae_loss_fwd: null pointer");
  EV_REQUIRE(B > 0 && P > 0 && L > 0 && L <= 256, "vae_loss_fwd: bad shape");
  hipLaunchKernelGGL(loss_fwd_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, x_hat, x, z, mu,
                     std, kl_lambda, elbo, kl, recon, P, L);
  hipLaunchKernelGGL(loss_mean_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, elbo, kl, recon,
                     loss, kl_loss, recon_loss, B);
  return evh::check_launch("vae_loss_fwd");
}

extern "C" int ebsdvae_vae_loss_bwd(const float* x_hat, const float* x, const float* z,
                                    const float* mu, const float* std, float kl_lambda,
                                    const float* g_loss, const float* g_kl_loss,
                                    const float* g_recon_loss, const float* g_elbo, float scale,
                                    float* g_xhat, float* g_z, float* g_mu, float* g_std,
                                    float* g_x, int B, int P, int L, ebsdvae_stream_t stream) {
  EV_REQUIRE(z && mu && std && g_z && g_mu && g_std && (!g_xhat || (x_hat && x)),
             "vae_loss_bwd: null pointer");
  EV_REQUIRE(B > 0 && P > 0 && L > 0 && L <= 256, "vae_loss_bwd: bad shape");
  const int bx = g_xhat ? (P / 4 + 255) / 256 + 1 : 1;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(bx, B), dim3(256), 0, (hipStream_t)stream, x_hat, x, z,
                     mu, std, kl_lambda, g_loss, g_kl_loss, g_recon_loss, g_elbo, scale, g_xhat,
                     g_z, g_mu, g_std, g_x, B, P, L);
  return evh::check_launch("vae_loss_bwd");
}

extern "C" int ebsdvae_vae_loss_fwd_parts(const float* bce_part, int tiles, const float* z,
                                          const float* mu, const float* std, float kl_lambda,
                                          float* elbo, float* kl, float* recon, float* loss,
                                          float* kl_loss, float* recon_loss, int B, int P, int L,
                                          ebsdvae_stream_t stream) {
  EV_REQUIRE(bce_part && z && mu && std && elbo && kl && recon && loss && kl_loss && recon_loss,
             "vae_loss_fwd_parts: null pointer");
  EV_REQUIRE(B > 0 && P > 0 && L > 0 && L <= 256 && tiles > 0, "vae_loss_fwd_parts: bad shape");
  hipLaunchKernelGGL(loss_fwd_parts_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, bce_part, tiles,
                     z, mu, std, kl_lambda, elbo, kl, recon, P, L);
  hipLaunchKernelGGL(loss_mean_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, elbo, kl, recon,
                     loss, kl_loss, recon_loss, B);
  return evh::check_launch("vae_loss_fwd_parts");
}
