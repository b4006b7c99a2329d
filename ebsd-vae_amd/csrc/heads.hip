// Latent heads, reparameterisation and sampler (latice/model.py:25-38, 55-64, 127-131).
//
//   flat   = encoder_out.flatten(1,-1)            NCHW order: k = c*S*S + h*S + w
//   mu     = flat @ Wmu^T + bmu ; logvar = flat @ Wlv^T + blv      (Linear(F, L))
//   std    = exp(logvar / 2) ;  z = mu + eps * std                (Normal(mu,std).rsample)
//   dec_in = (z @ W2^T + b2).view(B, C, S, S)   -> written NHWC for the decoder
//
// One 1024-thread workgroup per pattern (16 waves: the heads sit on the critical path
// between encoder and decoder, so latency matters more than the tiny FLOP count): the
// F-wide feature row lives in LDS, each thread dots its k-slice against every head row
// (coalesced weight rows), and the per-output sums fold through wave shuffles + LDS in a
// fixed order.  The NCHW<->NHWC flatten permutation is folded into the LDS index, so the
// NHWC encoder output never needs a transpose pass.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

constexpr int MAXL = 64;
constexpr int HT = 1024;         // threads per pattern
constexpr int HW_ = HT / 64;     // waves per pattern
constexpr int OCH = 32;          // head outputs per register chunk

// MU_ONLY: the encoder-only inference path (DiffractionPatternIndexer.build_dictionary
// consumes mu alone, latice/index/dp_indexer.py:136): only the mu head is evaluated.
template <bool MU_ONLY>
__global__ __launch_bounds__(HT) void heads_fwd_kernel(
    const float* __restrict__ enc, const float* __restrict__ wmu, const float* __restrict__ bmu,
    const float* __restrict__ wlv, const float* __restrict__ blv, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ eps, float* __restrict__ flat,
    float* __restrict__ mu, float* __restrict__ stdo, float* __restrict__ z,
    float* __restrict__ dec, int C, int S, int L) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int F = C * S * S;
  float* f = sm;                  // [F]
  float* red = sm + F;            // [HW_][2 * MAXL]
  float* zs = red + HW_ * 2 * MAXL;   // [MAXL]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* e = enc + (size_t)b * F;
  for (int i = tid; i < F; i += HT) {   // i = NHWC index within the pattern
    const int c = i % C, hw = i / C;
    f[c * S * S + hw] = e[i];
  }
  __syncthreads();
  if (!MU_ONLY)
    for (int k = tid; k < F; k += HT) flat[(size_t)b * F + k] = f[k];
  const int NO = MU_ONLY ? L : 2 * L;
  for (int o0 = 0; o0 < NO; o0 += OCH) {
    float acc[OCH];
#pragma unroll
    for (int j = 0; j < OCH; ++j) acc[j] = 0.f;
    for (int k = tid; k < F; k += HT) {
      const float fk = f[k];
#pragma unroll
      for (int j = 0; j < OCH; ++j) {
        const int o = o0 + j;
        if (o < NO) acc[j] = fmaf(fk, (o < L) ? wmu[(size_t)o * F + k] : wlv[(size_t)(o - L) * F + k], acc[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < OCH; ++j) {
      const float v = wave_sum(acc[j]);
      if (lane == 0 && o0 + j < NO) red[wave * 2 * MAXL + o0 + j] = v;
    }
  }
  __syncthreads();
  if (MU_ONLY) {
    if (tid < L) {
      float m = bmu[tid];
      for (int w = 0; w < HW_; ++w) m += red[w * 2 * MAXL + tid];
      mu[(size_t)b * L + tid] = m;
    }
    return;
  }
  if (tid < L) {
    float m = bmu[tid], lv = blv[tid];
    for (int w = 0; w < HW_; ++w) {
      m += red[w * 2 * MAXL + tid];
      lv += red[w * 2 * MAXL + L + tid];
    }
    const float sd = expf(lv * 0.5f);
    const float zz = fmaf(eps[(size_t)b * L + tid], sd, m);
    mu[(size_t)b * L + tid] = m;
    stdo[(size_t)b * L + tid] = sd;
    z[(size_t)b * L + tid] = zz;
    zs[tid] = zz;
  }
  __syncthreads();
  for (int o = tid; o < F; o += HT) {
    const float* wr = w2 + (size_t)o * L;
    float s = b2[o];
    for (int j = 0; j < L; ++j) s = fmaf(wr[j], zs[j], s);
    const int c = o / (S * S), hw = o - c * (S * S);
    dec[((size_t)b * S * S + hw) * C + c] = s;
  }
}

// gs layout per pattern: [g_mu_tot (L) | g_logvar (L) | g_out (F)]
__global__ __launch_bounds__(HT) void heads_bwd_kernel(
    const float* __restrict__ gdec, const float* __restrict__ gz, const float* __restrict__ gmu,
    const float* __restrict__ gstd, const float* __restrict__ stdv, const float* __restrict__ eps,
    const float* __restrict__ wmu, const float* __restrict__ wlv, const float* __restrict__ w2,
    float* __restrict__ genc, float* __restrict__ gs, int C, int S, int L) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int F = C * S * S;
  float* go = sm;                   // [F] g_out in flat (NCHW) order
  float* red = sm + F;              // [HW_][MAXL]
  float* gl = red + HW_ * MAXL;     // [2L]: g_mu_tot, g_logvar
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* gsb = gs + (size_t)b * (2 * L + F);
  for (int i = tid; i < F; i += HT) {
    const int c = i % C, hw = i / C;
    go[c * S * S + hw] = gdec[(size_t)b * F + i];
  }
  __syncthreads();
  for (int o = tid; o < F; o += HT) gsb[2 * L + o] = go[o];
  for (int j0 = 0; j0 < L; j0 += 16) {   // g_z[j] = sum_o g_out[o] * W2[o][j]
    float acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    for (int o = tid; o < F; o += HT) {
      const float g = go[o];
      const float* wr = w2 + (size_t)o * L + j0;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j0 + j < L) acc[j] = fmaf(g, wr[j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float v = wave_sum(acc[j]);
      if (lane == 0 && j0 + j < L) red[wave * MAXL + j0 + j] = v;
    }
  }
  __syncthreads();
  if (tid < L) {
    const int j = tid;
    const size_t bj = (size_t)b * L + j;
    float gzt = gz ? gz[bj] : 0.f;
    for (int w = 0; w < HW_; ++w) gzt += red[w * MAXL + j];
    const float sd = stdv[bj];
    const float gmt = gzt + (gmu ? gmu[bj] : 0.f);
    const float glv = ((gstd ? gstd[bj] : 0.f) + gzt * eps[bj]) * sd * 0.5f;
    gl[j] = gmt;
    gl[L + j] = glv;
    gsb[j] = gmt;
    gsb[L + j] = glv;
  }
  __syncthreads();
  for (int k = tid; k < F; k += HT) {
    float s = 0.f;
    for (int j = 0; j < L; ++j) {
      s = fmaf(gl[j], wmu[(size_t)j * F + k], s);
      s = fmaf(gl[L + j], wlv[(size_t)j * F + k], s);
    }
    const int c = k / (S * S), hw = k - c * (S * S);
    genc[((size_t)b * S * S + hw) * C + c] = s;
  }
}

// Weight grads of the three Linear layers as a split-batch reduction: blockIdx.y takes a
// chunk of HB patterns; thread (j, e) (e fastest: coalesced flat / g_out rows) writes its
// chunk's partial dWmu[j][e], dWlv[j][e], dW2[e][j] (stored [j][e]) and, for j == 0,
// db2[e]; threads past F*L take dbmu / dblv.  heads_wgrad_reduce sums the chunks in order.
constexpr int HB = 16;   // patterns per chunk

__global__ __launch_bounds__(256) void heads_wgrad_kernel(
    const float* __restrict__ flat, const float* __restrict__ z, const float* __restrict__ gs,
    float* __restrict__ part, int B, int F, int L) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int G = 2 * L + F;
  const size_t FL = (size_t)F * L;
  const size_t per = 3 * FL + F + 2 * L;   // one chunk's partial record
  float* pc = part + (size_t)blockIdx.y * per;
  const int b0 = blockIdx.y * HB, b1 = min(b0 + HB, B);
  if (idx < F * L) {
    const int j = idx / F, e = idx - j * F;
    float am = 0.f, al = 0.f, a2 = 0.f, ab = 0.f;
#pragma unroll 4
    for (int b = b0; b < b1; ++b) {
      const float fv = flat[(size_t)b * F + e];
      const float* gb = gs + (size_t)b * G;
      const float go = gb[2 * L + e];
      am = fmaf(gb[j], fv, am);
      al = fmaf(gb[L + j], fv, al);
      a2 = fmaf(go, z[(size_t)b * L + j], a2);
      ab += go;
    }
    pc[idx] = am;
    pc[FL + idx] = al;
    pc[2 * FL + idx] = a2;
    if (j == 0) pc[3 * FL + e] = ab;
  } else if (idx < F * L + L) {
    const int j = idx - F * L;
    float sm = 0.f, sl = 0.f;
    for (int b = b0; b < b1; ++b) {
      sm += gs[(size_t)b * G + j];
      sl += gs[(size_t)b * G + L + j];
    }
    pc[3 * FL + F + j] = sm;
    pc[3 * FL + F + L + j] = sl;
  }
}

__global__ __launch_bounds__(256) void heads_wgrad_reduce_kernel(
    const float* __restrict__ part, int nch, float* __restrict__ gwmu, float* __restrict__ gbmu,
    float* __restrict__ gwlv, float* __restrict__ gblv, float* __restrict__ gw2,
    float* __restrict__ gb2, int F, int L) {
  const size_t FL = (size_t)F * L;
  const size_t per = 3 * FL + F + 2 * L;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= per) return;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += part[(size_t)c * per + i];
  if (i < FL) {
    gwmu[i] = s;
  } else if (i < 2 * FL) {
    gwlv[i - FL] = s;
  } else if (i < 3 * FL) {
    const size_t r = i - 2 * FL;           // [j][e] -> W2 grad layout [e][j]
    const size_t j = r / F, e = r - j * F;
    gw2[e * L + j] = s;
  } else if (i < 3 * FL + F) {
    gb2[i - 3 * FL] = s;
  } else if (i < 3 * FL + F + L) {
    gbmu[i - 3 * FL - F] = s;
  } else {
    gblv[i - 3 * FL - F - L] = s;
  }
}

// ------------------------------------------------------------------ generic Linear
__global__ void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                  const float* __restrict__ b, float* __restrict__ y, int M, int K,
                                  int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= M * N) return;
  const int m = e / N, n = e - m * N;
  float s = b ? b[n] : 0.f;
  for (int k = 0; k < K; ++k) s = fmaf(x[(size_t)m * K + k], w[(size_t)n * K + k], s);
  y[e] = s;
}

__global__ void linear_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                  const float* __restrict__ gy, float* __restrict__ gx,
                                  float* __restrict__ gw, float* __restrict__ gb, int M, int K,
                                  int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = gx ? M * K : 0, nw = gw ? N * K : 0, nb = gb ? N : 0;
  if (e < nx) {
    const int m = e / K, k = e - m * K;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s = fmaf(gy[(size_t)m * N + n], w[(size_t)n * K + k], s);
    gx[e] = s;
  } else if (e < nx + nw) {
    const int i = e - nx, n = i / K, k = i - n * K;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s = fmaf(gy[(size_t)m * N + n], x[(size_t)m * K + k], s);
    gw[i] = s;
  } else if (e < nx + nw + nb) {
    const int n = e - nx - nw;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += gy[(size_t)m * N + n];
    gb[n] = s;
  }
}

__global__ void reparam_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                   const float* __restrict__ eps, float* __restrict__ z,
                                   float* __restrict__ sd, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = expf(lv[i] * 0.5f);
  if (sd) sd[i] = s;
  z[i] = fmaf(eps[i], s, mu[i]);
}

__global__ void reparam_bwd_kernel(const float* __restrict__ gz, const float* __restrict__ gsd,
                                   const float* __restrict__ eps, const float* __restrict__ sd,
                                   float* __restrict__ gmu, float* __restrict__ glv, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = gz ? gz[i] : 0.f;
  if (gmu) gmu[i] = g;
  if (glv) glv[i] = ((gsd ? gsd[i] : 0.f) + g * eps[i]) * sd[i] * 0.5f;
}

// ------------------------------------------------------------------ Philox4x32-10 normal
EV_DEVINL void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                            uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
  const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
  const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
  c0 = n0; c1 = l1; c2 = n2; c3 = l0;
}

__global__ void normal_tick_kernel(uint64_t* counter) { *counter += 1; }

__global__ void normal_fill_kernel(float* __restrict__ out, int64_t n, uint64_t seed,
                                   uint64_t offset, const uint64_t* __restrict__ counter) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;  // 4 normals per thread
  if (i * 4 >= n) return;
  const uint64_t base = counter ? offset + *counter * (uint64_t)((n + 3) / 4) : offset;
  const uint64_t ctr = base + (uint64_t)i;
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const float inv = 2.3283064365386963e-10f;  // 2^-32
  const float u0 = ((float)c0 + 0.5f) * inv, u1 = ((float)c1 + 0.5f) * inv;
  const float u2 = ((float)c2 + 0.5f) * inv, u3 = ((float)c3 + 0.5f) * inv;
  const float r0 = sqrtf(-2.f * logf(u0)), r1 = sqrtf(-2.f * logf(u2));
  const float tp = 6.283185307179586f;
  float v[4];
  v[0] = r0 * cosf(tp * u1);
  v[1] = r0 * sinf(tp * u1);
  v[2] = r1 * cosf(tp * u3);
  v[3] = r1 * sinf(tp * u3);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i * 4 + k < n) out[i * 4 + k] = v[k];
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_heads_fwd(const float* enc, const float* w_mu, const float* b_mu,
                                 const float* w_lv, const float* b_lv, const float* w_l2,
                                 const float* b_l2, const float* eps, float* flat, float* mu,
                                 float* std, float* z, float* dec_in, int B, int C, int S, int L,
                                 ebsdvae_stream_t stream) {
  EV_REQUIRE(enc && w_mu && b_mu && w_lv && b_lv && w_l2 && b_l2 && eps && flat && mu && std && z &&
                 dec_in,
             "heads_fwd: null pointer");
  EV_REQUIRE(B > 0 && L > 0 && L <= MAXL && C > 0 && S > 0, "heads_fwd: bad shape L=%d", L);
  const int F = C * S * S;
  const size_t lds = (F + (HW_ * 2 + 1) * MAXL) * sizeof(float);
  EV_REQUIRE(lds <= 160 * 1024, "heads_fwd: feature width %d too large", F);
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)heads_fwd_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(heads_fwd_kernel<false>, dim3(B), dim3(HT), lds, (hipStream_t)stream, enc, w_mu, b_mu,
                     w_lv, b_lv, w_l2, b_l2, eps, flat, mu, std, z, dec_in, C, S, L);
  return evh::check_launch("heads_fwd");
}

extern "C" int ebsdvae_latent_mu(const float* enc, const float* w_mu, const float* b_mu, float* mu,
                                 int B, int C, int S, int L, ebsdvae_stream_t stream) {
  EV_REQUIRE(enc && w_mu && b_mu && mu, "latent_mu: null pointer");
  EV_REQUIRE(B > 0 && L > 0 && L <= MAXL && C > 0 && S > 0, "latent_mu: bad shape L=%d", L);
  const int F = C * S * S;
  const size_t lds = (F + (HW_ * 2 + 1) * MAXL) * sizeof(float);
  EV_REQUIRE(lds <= 160 * 1024, "latent_mu: feature width %d too large", F);
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)heads_fwd_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(heads_fwd_kernel<true>, dim3(B), dim3(HT), lds, (hipStream_t)stream, enc, w_mu,
                     b_mu, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, mu, nullptr, nullptr,
                     nullptr, C, S, L);
  return evh::check_launch("latent_mu");
}

extern "C" int ebsdvae_heads_bwd(const float* g_dec, const float* g_z, const float* g_mu,
                                 const float* g_std, const float* std, const float* eps,
                                 const float* w_mu, const float* w_lv, const float* w_l2,
                                 float* g_enc, float* gs, int B, int C, int S, int L,
                                 ebsdvae_stream_t stream) {
  EV_REQUIRE(g_dec && std && eps && w_mu && w_lv && w_l2 && g_enc && gs, "heads_bwd: null pointer");
  EV_REQUIRE(B > 0 && L > 0 && L <= MAXL, "heads_bwd: bad shape");
  const int F = C * S * S;
  const size_t lds = (F + (HW_ + 2) * MAXL) * sizeof(float);
  EV_REQUIRE(lds <= 160 * 1024, "heads_bwd: feature width too large");
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)heads_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(heads_bwd_kernel, dim3(B), dim3(HT), lds, (hipStream_t)stream, g_dec, g_z, g_mu,
                     g_std, std, eps, w_mu, w_lv, w_l2, g_enc, gs, C, S, L);
  return evh::check_launch("heads_bwd");
}

extern "C" size_t ebsdvae_heads_wgrad_work(int B, int F, int L) {
  const size_t per = 3 * (size_t)F * L + F + 2 * (size_t)L;
  return (size_t)((B + HB - 1) / HB) * per * sizeof(float);
}

extern "C" int ebsdvae_heads_wgrad(const float* flat, const float* z, const float* gs, float* gw_mu,
                                   float* gb_mu, float* gw_lv, float* gb_lv, float* gw_l2,
                                   float* gb_l2, void* work, int B, int F, int L,
                                   ebsdvae_stream_t stream) {
  EV_REQUIRE(flat && z && gs && gw_mu && gb_mu && gw_lv && gb_lv && gw_l2 && gb_l2 && work,
             "heads_wgrad: null pointer");
  EV_REQUIRE(B > 0 && L > 0 && L <= MAXL, "heads_wgrad: bad L");
  const int n = F * L + L;
  const int nch = (B + HB - 1) / HB;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(heads_wgrad_kernel, dim3((n + 255) / 256, nch), dim3(256), 0, s, flat, z, gs,
                     (float*)work, B, F, L);
  const size_t per = 3 * (size_t)F * L + F + 2 * (size_t)L;
  hipLaunchKernelGGL(heads_wgrad_reduce_kernel, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, s,
                     (const float*)work, nch, gw_mu, gb_mu, gw_lv, gb_lv, gw_l2, gb_l2, F, L);
  return evh::check_launch("heads_wgrad");
}

extern "C" int ebsdvae_linear_fwd(const float* x, const float* w, const float* b, float* y, int M,
                                  int K, int N, ebsdvae_stream_t stream) {
  EV_REQUIRE(x && w && y && M > 0 && K > 0 && N > 0, "linear_fwd: bad args");
  const int n = M * N;
  hipLaunchKernelGGL(linear_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, w,
                     b, y, M, K, N);
  return evh::check_launch("linear_fwd");
}

extern "C" int ebsdvae_linear_bwd(const float* x, const float* w, const float* gy, float* gx,
                                  float* gw, float* gb, int M, int K, int N,
                                  ebsdvae_stream_t stream) {
  EV_REQUIRE(x && w && gy && M > 0 && K > 0 && N > 0, "linear_bwd: bad args");
  const int n = (gx ? M * K : 0) + (gw ? N * K : 0) + (gb ? N : 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(linear_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, w,
                     gy, gx, gw, gb, M, K, N);
  return evh::check_launch("linear_bwd");
}

extern "C" int ebsdvae_reparam_fwd(const float* mu, const float* logvar, const float* eps, float* z,
                                   float* std, int64_t n, ebsdvae_stream_t stream) {
  EV_REQUIRE(mu && logvar && eps && z && n >= 0, "reparam_fwd: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(reparam_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, mu, logvar, eps, z, std, n);
  return evh::check_launch("reparam_fwd");
}

extern "C" int ebsdvae_reparam_bwd(const float* gz, const float* gstd, const float* eps,
                                   const float* std, float* gmu, float* glogvar, int64_t n,
                                   ebsdvae_stream_t stream) {
  EV_REQUIRE(eps && std && n >= 0, "reparam_bwd: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(reparam_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gz, gstd, eps, std, gmu, glogvar, n);
  return evh::check_launch("reparam_bwd");
}

extern "C" int ebsdvae_normal_fill(float* out, int64_t n, uint64_t seed, uint64_t offset,
                                   uint64_t* counter, ebsdvae_stream_t stream) {
  EV_REQUIRE(out && n >= 0, "normal_fill: bad args");
  if (n == 0) return 0;
  const int64_t threads = (n + 3) / 4;
  if (counter) hipLaunchKernelGGL(normal_tick_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
  hipLaunchKernelGGL(normal_fill_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, out, n, seed, offset, counter);
  return evh::check_launch("normal_fill");
}
