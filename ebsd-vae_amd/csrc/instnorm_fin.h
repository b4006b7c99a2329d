// InstanceNorm finalize steps shared by the standalone kernels (instnorm.hip) and the
// persistent split conv, which runs them for the images it owns after its last tile
// (conv_split.hip): one image b per call, 256 active threads, the same summation order in
// both places (bit-identical results).  Every thread of the block calls them (they contain
// workgroup barriers); threads with tid >= 256 only take part in the barriers.
#pragma once
#include "common.h"

namespace ev {

// Forward statistics {mean, rstd} of image b from T per-tile {mean, M2} partials of n pixels
// each: thread (c = tid % C, j = tid / C) folds tiles j, j+J, ... of channel c (coalesced over
// c), then lane j == 0 folds the J partial results in order.  All tiles hold n elements, so
// the Chan merge reduces to mean = avg(mean_t), M2 = sum(M2_t) + n * sum((mean_t - mean)^2).
// sm: 3 x 256 floats of LDS.
EV_DEVINL void in_stats_finalize_image(const float2* __restrict__ part, float2* __restrict__ st,
                                       int C, int T, float n, int b, int tid, float* sm) {
  const bool on = tid < 256;
  const int J = 256 / C;
  const int c = tid % C, j = tid / C;
  const float2* p = part + (size_t)b * T * C + c;
  float m = 0.f;
  if (on) {
#pragma unroll 8
    for (int t = j; t < T; t += J) m += p[(size_t)t * C].x;
    sm[tid] = m;
  }
  __syncthreads();
  float mean = 0.f, m2 = 0.f, dm = 0.f;
  if (on) {
    for (int k = 0; k < J; ++k) mean += sm[k * C + c];
    mean /= (float)T;
#pragma unroll 8
    for (int t = j; t < T; t += J) {
      const float2 v = p[(size_t)t * C];
      m2 += v.y;
      const float d = v.x - mean;
      dm = fmaf(d, d, dm);
    }
  }
  __syncthreads();
  if (on) {
    sm[tid] = m2;
    sm[512 + tid] = dm;
  }
  __syncthreads();
  if (on && j == 0) {
    float a = 0.f, q = 0.f;
    for (int k = 0; k < J; ++k) { a += sm[k * C + c]; q += sm[512 + k * C + c]; }
    const float var = (a + n * q) / (n * (float)T);
    st[(size_t)b * C + c] = make_float2(mean, 1.0f / sqrtf(var + kInEps));
  }
  __syncthreads();   // sm is free again on return
}

// InstanceNorm-backward statistics of image b: {mean(g_xhat), mean(g_xhat * xhat)} from T
// per-tile double sums (C <= 256): thread (c, j) sums tiles j, j+J, ... of channel c in
// double, then lane j == 0 folds the J sums in order.  sm: 2 x 256 doubles of LDS.
EV_DEVINL void in_bwd_finalize_image(const double2* __restrict__ part, float2* __restrict__ bst,
                                     int C, int T, double inv_hw, int b, int tid, double* sm) {
  const bool on = tid < 256;
  const int J = 256 / C;
  const int c = tid % C, j = tid / C;
  const double2* p = part + (size_t)b * T * C + c;
  if (on) {
    double s1 = 0.0, s2 = 0.0;
    if (j < J) {
#pragma unroll 8
      for (int t = j; t < T; t += J) {
        const double2 v = p[(size_t)t * C];
        s1 += v.x;
        s2 += v.y;
      }
    }
    sm[tid] = s1;
    sm[256 + tid] = s2;
  }
  __syncthreads();
  if (on && j == 0) {
    double a = 0.0, q = 0.0;
    for (int k = 0; k < J; ++k) { a += sm[k * C + c]; q += sm[256 + k * C + c]; }
    bst[(size_t)b * C + c] = make_float2((float)(a * inv_hw), (float)(q * inv_hw));
  }
  __syncthreads();
}

}  // namespace ev
