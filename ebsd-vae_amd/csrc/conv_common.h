// Pieces shared by the fp32 (conv_fwd.hip) and split-bf16 (conv_x3.hip) implicit-GEMM
// conv kernels: the LDS DMA helper, the epilogue (bias, y stores, InstanceNorm partials)
// and the fused InstanceNorm-backward reduce of input-gradient launches.  Both MFMA
// families write the same 32x32 accumulator layout (col = lane & 31, row = (r & 3) +
// 8 (r >> 2) + 4 (lane >> 5)), so one epilogue serves both.
#pragma once
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

typedef __attribute__((address_space(3))) void* lds_void_ptr;

EV_DEVINL void glds16(const float* g, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void*)g, (lds_void_ptr)lds_wave_base, 16, 0, 0);
}

// ------------------------------------------------------------------ shared epilogue
constexpr int FP_NONE = -1;   // no fused InstanceNorm-backward reduce
// forward of a layer whose output the next layer max-pools (pipelined split kernel only):
// the epilogue also writes the 2x2 max of the raw output y at (H/2, W/2)
constexpr int FP_POOLOUT = 3;
// input gradient whose consumer upsampled its source (pmode P_UPSUM at the ABI): the
// epilogue writes the 2x2 window sums (the gradient w.r.t. the pre-upsample activation, at
// (H/2, W/2)) instead of the full-resolution gradient, and fuses the previous block's
// InstanceNorm-backward reduce per window
constexpr int FP_UPSUM = 4;

// Fused InstanceNorm-backward reduce of the PREVIOUS block (input-gradient convs only):
// this conv's product is g = d loss / d a_prev (a_prev = [pool|up](lrelu(IN(y_prev))) at
// this conv's resolution).  Per element it adds h = g * lrelu'(xhat) and h * xhat of
// the y_prev pixel that g routes to (identity, the 2x2 argmax, or the upsample parent)
// -- the sums ebsdvae_in_bwd_reduce would compute, without re-reading g -- and the conv
// writes h, not g: every consumer of a fused input gradient (the InstanceNorm-backward
// apply, the first block's pass, the gy-staging input-gradient conv) needs h, and the
// LeakyReLU branch is then taken once, where the reduce takes it.
// y_prev offset (in pixels of y_prev) of the k-th value read for conv pixel pl
template <int FP>
EV_DEVINL int inbwd_pix(int pl, int W, int lW, int k) {
  const int h = pl >> lW, w = pl & (W - 1);
  if (FP == P_ID) return pl;
  if (FP == P_UP) return (h >> 1) * (W >> 1) + (w >> 1);
  return (2 * h + (k >> 1)) * (2 * W) + 2 * w + (k & 1);   // P_POOL window (k = dy*2+dx)
}

// sp = {mean, rstd} of the y_prev channel; c = -mean * rstd.  Identity / upsample routing: the
// LeakyReLU branch is y > mean -- exactly the sign of (y - mean) * rstd (rstd > 0, no
// underflow), which the pinned oracle evaluates -- and xhat, which only enters the second sum,
// is one fma.  The 2x2 argmax compares lrelu((y - mean) * rstd) as the reference's pool does.
template <int FP>
EV_DEVINL float inbwd_acc(float g, const float* v, float2 sp, float c, float& s1, float& s2) {
  float ga, x;
  if (FP == P_POOL) {   // first maximum of lrelu(xhat) in window order (0,0),(0,1),(1,0),(1,1)
    x = (v[0] - sp.x) * sp.y;
    float best = lrelu(x);
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float xk = (v[k] - sp.x) * sp.y;
      const float f = lrelu(xk);
      if (f > best) { best = f; x = xk; }
    }
    ga = g * slope(x);
  } else {
    x = fmaf(v[0], sp.y, c);
    ga = v[0] > sp.x ? g : g * kSlope;
  }
  s1 += ga;
  s2 = fmaf(ga, x, s2);
  return ga;
}

template <int MF, int NF, int FP, int GMAX = 32>
EV_DEVINL void conv_epilogue(f32x16 (&acc)[MF][NF], const float* __restrict__ bias,
                             float* __restrict__ y, float2* __restrict__ spart, int B, int H,
                             int W, int Cout, int b0, int h0, int tpx, int wpx0, int co_base,
                             int hk, int l32, const float* __restrict__ yprev,
                             const float2* __restrict__ stprev, double2* __restrict__ ipart) {
  constexpr int MW = MF * 32;
  const int wimg = wpx0 / tpx;  // the wave's pixels lie in ONE image
  const int gb = b0 + wimg;
  const bool bvalid = gb < B;
  const int T = (H * W) / MW;
  const int slot = (h0 * W + (wpx0 - wimg * tpx)) / MW;
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int co = co_base + nf * 32 + l32;
    const float bb = bias ? bias[co] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wpx0 + mf * 32 + (r & 3) + 8 * (r >> 2) + 4 * hk;
        const int rem = m - wimg * tpx;
        const float v = acc[mf][nf][r] + bb;
        acc[mf][nf][r] = v;
        s += v;
        // a fused input gradient writes h (below), the forward its pre-norm output
        if (FP == FP_NONE && bvalid) y[(((size_t)gb * H + h0) * W + rem) * Cout + co] = v;
      }
    if (FP != FP_NONE && bvalid) {
      // loads in batches of GMAX values issued before any use (latency overlapped within a batch)
      constexpr int NL = FP == P_POOL ? 4 : 1;
      constexpr int G = (GMAX / NL) < MF * 16 ? (GMAX / NL) : MF * 16;
      static_assert((MF * 16) % G == 0, "batch size");
      const int lW = 31 - __builtin_clz(W);
      const size_t plane = FP == P_POOL ? (size_t)4 * H * W : (FP == P_UP ? (size_t)(H * W) / 4 : (size_t)H * W);
      const float* yp = yprev + (size_t)gb * plane * Cout + co;
      const float2 sp = stprev[(size_t)gb * Cout + co];
      const float sc = -sp.x * sp.y;
      const int pbase = h0 * W - wimg * tpx + wpx0 + 4 * hk;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e0 = 0; e0 < MF * 16; e0 += G) {
        float v[G][NL];
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int e = e0 + j, mf = e >> 4, r = e & 15;
          const int pl = pbase + mf * 32 + (r & 3) + 8 * (r >> 2);
#pragma unroll
          for (int k = 0; k < NL; ++k) v[j][k] = yp[(size_t)inbwd_pix<FP>(pl, W, lW, k) * Cout];
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int e = e0 + j, mf = e >> 4, r = e & 15;
          const float h = inbwd_acc<FP>(acc[mf][nf][r], v[j], sp, sc, s1, s2);
          const int rem = wpx0 + mf * 32 + (r & 3) + 8 * (r >> 2) + 4 * hk - wimg * tpx;
          y[(((size_t)gb * H + h0) * W + rem) * Cout + co] = h;
        }
      }
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (hk == 0) ipart[((size_t)gb * T + slot) * Cout + co] = make_double2((double)s1, (double)s2);
    }
    if (spart) {
      s += __shfl_xor(s, 32, 64);
      const float mean = s * (1.0f / MW);
      float q = 0.f;
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[mf][nf][r] - mean;
          q = fmaf(d, d, q);
        }
      q += __shfl_xor(q, 32, 64);
      if (hk == 0 && bvalid) spart[((size_t)gb * T + slot) * Cout + co] = make_float2(mean, q);
    }
  }
}


// batched weight-pack descriptors, passed to the pack kernels by value
struct PackBatch {
  ebsdvae_pack_desc d[EBSDVAE_MAX_PACK];
};

// fused InstanceNorm-backward reduce arguments of input-gradient launches (FP != FP_NONE)
struct InBwdFuse {
  const float* yprev = nullptr;
  const float2* stprev = nullptr;
  double2* part = nullptr;
  float* ypool = nullptr;   // FP_POOLOUT forward: the max-pooled raw output
  const float* gmax = nullptr;   // NP_F16 input gradient: per-tile max |g| (B, gmT)
  int gmT = 0;
  float2* st_out = nullptr;      // in-kernel InstanceNorm finalize (pipe_owns_images): forward
  float2* bst_out = nullptr;     // {mean, rstd}, or the previous block's backward {m1, m2}
  double inv_hw = 0.0;           // 1 / (H*W) of the previous block (bst_out)
  const float* w0 = nullptr;     // ACT_FIRST forward: the first conv's weight (cin,1,3,3) and
  const float* b0 = nullptr;     // bias, which the staging recomputes y0 from x with
};

}  // namespace ev
