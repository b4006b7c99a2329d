// Network end of the training step in ONE pass over the last block's pre-norm output y13:
//   x_hat = Conv2d(32, 1)(lrelu(IN(y13)))                        latice/model.py:147-148
//   BCE-with-logits per-sample sums, and its logit gradient       lightning_module.py:79-92
//     g1 = d loss / d x_hat = g_loss * scale / (B * P) * (sigmoid(x_hat) - x)
//   the InstanceNorm-backward reduce of that block (sum g_a*lrelu', sum g_a*lrelu'*xhat per
//   (b, c), g_a = the final conv's input gradient recomputed from g1) and the final conv's
//   weight / bias gradient partials                                (autograd of :147-148)
// These were three kernels that each read y13 (512 MB at B = 256): the 32 -> 1 conv, the loss
// (x_hat, x) and the fused final reduce (in_bwd_edge_kernel<FUSE_FINAL, false>).  The apply
// pass that writes the block's output gradient (ebsdvae_in_bwd_final_apply_max) reads g1 from
// here and is unchanged.
//
// Block = one band of TH output rows of one image (W = 128 or 256: 8 channel groups x W/4 pixel
// lanes, 4 pixels per thread per row; 256 or 512 threads).  It streams the source rows
// r0-2 .. r0+TH+1 once: row q is normalised to a = lrelu(IN(y13)) (registers, three rows deep)
// and contracted with the nine taps into a 4-row ring of tap planes in LDS; x_hat / g1 of row
// q-1 follow from the planes (g1 into a 4-row ring); the reduce of row q-2 from the g1 ring and
// the registers' a.  Four slots let every step write the slot of a row the previous step no
// longer reads, so two barriers per row suffice.  The two halo rows above and below are
// recomputed by the neighbouring bands (x_hat / g1 are written only for the band's own rows).
// The sums are fp32 per row and thread, double across rows, lanes and waves (fixed order), as
// the reduce kernel it replaces.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

// rows per band: the two recomputed halo rows above and below cost 4 / TH of the band's work
// band rows: 64 where H allows (round 6: the recomputed halo rows are 6 of every 70 steps
// instead of 6 of 38), else 32
#ifndef EV_NE_TH
#define EV_NE_TH 64
#endif
constexpr int NE_C = 32, NE_TH = EV_NE_TH, NE_TH_MIN = 32;
#ifndef EV_NE_FOLD
#define EV_NE_FOLD 8
#endif
constexpr int NE_FOLD = EV_NE_FOLD;   // rows per running sum of net_end_mfma_kernel (power of two)
constexpr int ne_th(int H) { return H % NE_TH == 0 ? NE_TH : NE_TH_MIN; }
constexpr int NE_RING = 4;
#ifndef EV_NE_UNROLL6
#define EV_NE_UNROLL6 1
#endif
#ifndef EV_NE_BRFREE
#define EV_NE_BRFREE 1
#endif                 // ring slots (a and g1): slot(row) = (row - r0 + k) & 3
// per width: threads, ring row (zero column, W pixels, zero column)
template <int W> constexpr int ne_nth() { return 2 * W; }
template <int W> constexpr int ne_wp() { return W + 2; }

// BCE-with-logits term and sigmoid from one e = exp(-|x|) and one division: the same values as
//   (1 - t) x + max(-x, 0) + log1p(exp(-|x|))  and  x >= 0 ? 1 / (1 + exp(-x)) : exp(x) / (1 + exp(x))
EV_DEVINL float ne_bce_e(float xh, float t, float e) { return (1.f - t) * xh + fmaxf(-xh, 0.f) + log1pf(e); }
EV_DEVINL float ne_sigmoid_e(float x, float e) { return (x >= 0.f ? 1.f : e) / (1.f + e); }
// sum over the 8 channel-group lanes of a pixel (lanes 8k .. 8k+7), on the VALU through DPP:
// quad_perm [1,0,3,2] (xor 1), [2,3,0,1] (xor 2), then row_half_mirror (lane i <-> 7 - i,
// which pairs the two quads of the 8-lane group)
template <int CTRL>
EV_DEVINL float ne_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
EV_DEVINL float ne_fold8(float v) {
  v += ne_dpp<0xB1>(v);
  v += ne_dpp<0x4E>(v);
  v += ne_dpp<0x141>(v);
  return v;
}


// u-ring: the nine tap planes of one source row, u_t[w] = sum_c a[w][c] * w14[c][t] (zero
// columns at w = -1 and w = W), so x_hat[r][w] = b14 + sum_t u_t(row r - 1 + kh)[w - 1 + kw]
template <int W> constexpr int ne_urow() { return 9 * (W + 2); }
template <int W> constexpr size_t ne_lds_u() {
  return (size_t)(NE_RING * ne_urow<W>() + NE_RING * ne_wp<W>()) * sizeof(float);
}

// a * (w.x, w.x) + c and a * (w.y, w.y) + c: one half of a packed weight pair broadcast by the
// op_sel modifiers (written as pk2(w.x, w.x), hipcc materialises the 36 broadcast pairs as
// loop-invariant registers and spills them)
EV_DEVINL pkf2 ne_fma_wx(pkf2 a, pkf2 w, pkf2 c) {
  pkf2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  return d;
}
EV_DEVINL pkf2 ne_fma_wy(pkf2 a, pkf2 w, pkf2 c) {
  pkf2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(d) : "v"(a), "v"(w), "v"(c));
  return d;
}

// lanes cg ^ 4, cg ^ 2, cg ^ 1 of the 8-lane channel group (DPP row_half_mirror pairs lane i
// with 7 - i: bit 2 differs; quad_perm [2,3,0,1] / [1,0,3,2])
EV_DEVINL float ne_x4(float v) { return ne_dpp<0x141>(v); }
EV_DEVINL float ne_x2(float v) { return ne_dpp<0x4E>(v); }
EV_DEVINL float ne_x1(float v) { return ne_dpp<0xB1>(v); }

// Round 5: the final conv's channel contraction without an activation ring.  Each thread
// contracts its own 4 channels of a = lrelu(IN(y13)) with the 9 taps for its 4 pixels (the
// values stay in registers, 3 rows deep, for the reduce), the 8 channel-group lanes of a pixel
// combine their partials by a DPP reduce-scatter (lane cg ends with pixel 2 (cg >> 2) +
// ((cg >> 1) & 1)'s sums for taps 0-4 or 5-8), and those go to a 4-row ring of tap planes.
// x_hat then needs 9 scalar reads per pixel instead of 9 16-byte activation reads per
// (pixel, channel group), and the reduce reads its activation from registers: round 4's
// activation-ring kernel moved 784 B of LDS per thread and row, this one 180.  Measured (PMC,
// B = 256): 207 vs 216 us -- both are VALU-issue-bound (668 VALU per wave and row, 216 of them
// the three 288-MAC-per-pixel contractions), not LDS-bound.
template <int W, int TH>
__global__ __launch_bounds__(ne_nth<W>(), W == 128 ? 2 : 1) void net_end_kernel(
    const float* __restrict__ y, const float2* __restrict__ st, const float* __restrict__ w14,
    const float* __restrict__ b14, const float* __restrict__ xt, const float* __restrict__ g_loss,
    float gscale, float* __restrict__ x_hat, float* __restrict__ g1out, float* __restrict__ bce_part,
    double2* __restrict__ part, float* __restrict__ wpart, float* __restrict__ bpart, int H) {
  constexpr int C = NE_C, WP = ne_wp<W>(), UROW = ne_urow<W>();
  constexpr int NE_NTH = ne_nth<W>(), NPL = W / 4, NWAVE = NE_NTH / 64;
  extern __shared__ __attribute__((aligned(16))) float ne_sm[];
  float* uring = ne_sm;                       // [4][9][WP]
  float* gring = ne_sm + NE_RING * UROW;      // [4][WP]
  const int tile = blockIdx.x, b = blockIdx.y, T = gridDim.x;
  const int tid = threadIdx.x, cg = tid & 7, pl = tid >> 3;
  const int c = cg * 4;
  const int r0 = tile * TH;
  const size_t HW = (size_t)H * W;

  float2 fs[4];   // {rstd, -mean * rstd}
#pragma unroll
  for (int k = 0; k < 4; ++k) fs[k] = norm_fs(st[(size_t)b * C + c + k]);
  const pkf2 fsr[2] = {pk2(fs[0].x, fs[1].x), pk2(fs[2].x, fs[3].x)};   // rstd pairs
  const pkf2 fsb[2] = {pk2(fs[0].y, fs[1].y), pk2(fs[2].y, fs[3].y)};   // -mean * rstd pairs
  pkf2 wv2[2][9];   // w14 (1, 32, 3, 3) as channel pairs (c, c+1), (c+2, c+3)
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t) wv2[k][t] = pk2(w14[(c + 2 * k) * 9 + t], w14[(c + 2 * k + 1) * 9 + t]);
  const float bias = b14 ? b14[0] : 0.f;
  const float cr = gscale * (g_loss ? *g_loss : 1.f);   // g_loss * scale / (B * P)

  // zero columns of both rings (never written by the row passes)
  for (int i = tid; i < NE_RING * 9 * 2; i += NE_NTH) {
    const int r = i / 18, t = (i >> 1) % 9, side = i & 1;
    uring[r * UROW + t * WP + side * (W + 1)] = 0.f;
  }
  if (tid < 2 * NE_RING) gring[(tid >> 1) * WP + (tid & 1) * (W + 1)] = 0.f;

  const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + (size_t)b * HW * C), 0,
                                                    (int)(HW * C * 4), 0x00020000);
  auto load_row = [&](int q, float4 (&d)[4]) EV_LAMBDA_INLINE {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      d[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                            ry, ((q * W + pl + NPL * j) * C + c) * 4, 0, 0));
  };

  double s1d[4] = {0.0, 0.0, 0.0, 0.0}, s2d[4] = {0.0, 0.0, 0.0, 0.0};
  pkf2 wacc2[2][9];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t) wacc2[k][t] = pk2(0.f, 0.f);
  float bsum = 0.f, bce = 0.f;
  auto load_tgt = [&](int r, float& d) EV_LAMBDA_INLINE {
    d = (r >= 0 && r < H && cg < 4) ? xt[(size_t)b * HW + (size_t)r * W + pl + NPL * cg] : 0.f;
  };
  float4 ybuf[2][4];
  float tbuf[2];
  float4 am1[4], am2[4];   // a of source rows q - 1, q - 2 (this thread's pixels and channels)
#pragma unroll
  for (int j = 0; j < 4; ++j) am1[j] = am2[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  load_row(r0 - 2, ybuf[0]);
  load_row(r0 - 1, ybuf[1]);
  load_tgt(r0 - 3, tbuf[0]);
  load_tgt(r0 - 2, tbuf[1]);
  // this lane's share after the reduce-scatter: pixel jk of the thread's four, taps t0 .. t0+nt-1
  const int jk = 2 * (cg >> 2) + ((cg >> 1) & 1);
  const bool hi4 = cg & 4, hi2 = cg & 2, hi1 = cg & 1;
  __syncthreads();   // ring columns zeroed

  auto step = [&](int i, float4 (&ycur)[4], float& tcur) EV_LAMBDA_INLINE {
    const int q = r0 - 2 + i;
    // (1) a of source row q (registers), its tap contraction into ring slot i & 3
    float4 aq[4];
    if (q >= 0 && q < H) {   // block-uniform
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 v = ycur[j];
        const pkf2 u0 = pkfma(pk2(v.x, v.y), fsr[0], fsb[0]), u1 = pkfma(pk2(v.z, v.w), fsr[1], fsb[1]);
        const pkf2 k0 = u0 * pk2(kSlope, kSlope), k1 = u1 * pk2(kSlope, kSlope);
        aq[j] = make_float4(fmaxf(u0.x, k0.x), fmaxf(u0.y, k0.y), fmaxf(u1.x, k1.x), fmaxf(u1.y, k1.y));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) aq[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    load_row(q + 2, ycur);   // prefetch into the registers just consumed
    {
      // partial u over this lane's 4 channels, pixels paired (j, j + 1) per packed fma
      pkf2 up[2][9];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 A = aq[2 * h], Bv = aq[2 * h + 1];
        const pkf2 ch[4] = {pk2(A.x, Bv.x), pk2(A.y, Bv.y), pk2(A.z, Bv.z), pk2(A.w, Bv.w)};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          pkf2 a2 = ne_fma_wx(ch[0], wv2[0][t], pk2(0.f, 0.f));
          a2 = ne_fma_wy(ch[1], wv2[0][t], a2);
          a2 = ne_fma_wx(ch[2], wv2[1][t], a2);
          up[h][t] = ne_fma_wy(ch[3], wv2[1][t], a2);
        }
      }
      // reduce-scatter over the 8 channel-group lanes: pixels {0,1} | {2,3} by bit 2 ...
      float r1[2][9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float k0 = hi4 ? up[1][t].x : up[0][t].x, k1 = hi4 ? up[1][t].y : up[0][t].y;
        const float s0 = hi4 ? up[0][t].x : up[1][t].x, s1 = hi4 ? up[0][t].y : up[1][t].y;
        r1[0][t] = k0 + ne_x4(s0);
        r1[1][t] = k1 + ne_x4(s1);
      }
      // ... one pixel by bit 1 ...
      float r2[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float k = hi2 ? r1[1][t] : r1[0][t], sd = hi2 ? r1[0][t] : r1[1][t];
        r2[t] = k + ne_x2(sd);
      }
      // ... taps 0-4 | 5-8 by bit 0 (tap 4 sent by the bit-1 lane, whose share is 5-8)
      float r3[5];
#pragma unroll
      for (int e = 0; e < 5; ++e) {
        const float k = hi1 ? (e < 4 ? r2[5 + e] : 0.f) : r2[e];
        const float sd = hi1 ? r2[e] : (e < 4 ? r2[5 + e] : 0.f);
        r3[e] = k + ne_x1(sd);
      }
      float* ur = uring + (i & 3) * UROW + pl + NPL * jk + 1;
#pragma unroll
      for (int e = 0; e < 5; ++e)
        if (!hi1 || e < 4) ur[(hi1 ? 5 + e : e) * WP] = r3[e];
    }
    __syncthreads();
    // (2) x_hat, g1 and BCE of row q - 1 from the tap planes of rows q - 2, q - 1, q
    if (i >= 2) {
      const int r = q - 1;
      const bool inrow = r >= 0 && r < H, own = r >= r0 && r < r0 + TH;
      float* gr = gring + (i & 3) * WP;   // g1 row r0 - 3 + i
      if (cg < 4) {
        const int w = pl + NPL * cg;
        float xh = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const float* u = uring + ((i - 2 + kh) & 3) * UROW + w;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) xh += u[(kh * 3 + kw) * WP + kw];
        }
        xh += bias;
        float g = 0.f;
        if (inrow) {
          const float e = expf(-fabsf(xh));
          g = cr * (ne_sigmoid_e(xh, e) - tcur);
          if (own) {
            x_hat[(size_t)b * HW + (size_t)r * W + w] = xh;
            g1out[(size_t)b * HW + (size_t)r * W + w] = g;
            bce += ne_bce_e(xh, tcur, e);
            bsum += g;
          }
        }
        gr[w + 1] = g;
      }
    }
    load_tgt(q + 1, tcur);   // x_hat row q + 1 is computed at step i + 2
    __syncthreads();
    // (3) InstanceNorm-backward reduce + final-conv weight gradient of row q - 2 (a in am2)
    if (i >= 4) {
      const float* gA = gring + ((i - 2) & 3) * WP;        // row q - 3
      const float* gB = gring + ((i - 1) & 3) * WP;        // row q - 2
      const float* gC = gring + (i & 3) * WP;              // row q - 1
      pkf2 s1[2] = {pk2(0.f, 0.f), pk2(0.f, 0.f)}, s2[2] = {pk2(0.f, 0.f), pk2(0.f, 0.f)};
#pragma unroll   // am2[j]: registers only with a constant index
      for (int j = 0; j < 4; ++j) {
        const int w = pl + NPL * j;
        float nb[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int kh = t / 3, kw = t % 3;
          const float* grw = kh == 0 ? gC : (kh == 1 ? gB : gA);
          nb[t] = grw[w + 2 - kw];
        }
        pkf2 ga[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          pkf2 sg = pk2(0.f, 0.f);
#pragma unroll
          for (int t = 0; t < 9; ++t) sg = pkfma(pk2(nb[t], nb[t]), wv2[k][t], sg);
          ga[k] = sg;
        }
        const float4 a4 = am2[j];
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const pkf2 a2 = pk2(av[2 * k], av[2 * k + 1]);
          const pkf2 xs = a2 * pk2(1.f / kSlope, 1.f / kSlope);
          const bool p0 = a2.x > 0.f, p1 = a2.y > 0.f;
          const pkf2 xh = pk2(p0 ? a2.x : xs.x, p1 ? a2.y : xs.y);
          const pkf2 gx = ga[k] * pk2(p0 ? 1.f : kSlope, p1 ? 1.f : kSlope);
          s1[k] += gx;
          s2[k] = pkfma(gx, xh, s2[k]);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const pkf2 f = pk2(av[2 * k], av[2 * k + 1]);
#pragma unroll
          for (int t = 0; t < 9; ++t) wacc2[k][t] = pkfma(pk2(nb[t], nb[t]), f, wacc2[k][t]);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        s1d[k] += (double)((k & 1) ? s1[k >> 1].y : s1[k >> 1].x);
        s2d[k] += (double)((k & 1) ? s2[k >> 1].y : s2[k >> 1].x);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { am2[j] = am1[j]; am1[j] = aq[j]; }
  };
#pragma unroll 1
  for (int i = 0; i < TH + 4; i += 2) {
    step(i, ybuf[0], tbuf[0]);
    step(i + 1, ybuf[1], tbuf[1]);
  }
  __syncthreads();
  // ---- band partials, fixed order: lanes of a channel group in-wave, then the NWAVE waves
  const int lane = tid & 63, wave = tid >> 6;
  // (a tree of lane shuffles: a serial 32-step LDS walk here cost ~8 us per block)
  double* red = reinterpret_cast<double*>(ne_sm);            // [NWAVE][8 cg][8]
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    double v = k < 4 ? s1d[k] : s2d[k - 4];
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 8) red[(wave * 8 + lane) * 8 + k] = v;
  }
  __syncthreads();
  const int slice = b * T + tile;
  if (tid < C) {   // channel c = tid: group tid / 4, element tid % 4
    const int g = tid >> 2, k = tid & 3;
    double u = 0.0, v = 0.0;
#pragma unroll
    for (int wv = 0; wv < NWAVE; ++wv) { u += red[(wv * 8 + g) * 8 + k]; v += red[(wv * 8 + g) * 8 + 4 + k]; }
    part[(size_t)slice * C + tid] = make_double2(u, v);
  }
  __syncthreads();
  // weight-gradient partials [slice][tap][0][ci]: fold the 32 pixel lanes of each channel group
  float* wred = ne_sm;   // [NWAVE][8 cg][36 + 2]
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float v = (k & 1) ? wacc2[k >> 1][t].y : wacc2[k >> 1][t].x;
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 8) wred[(wave * 8 + lane) * 38 + k * 9 + t] = v;
    }
  {
    float v = bsum, e = bce;   // lanes cg < 4 hold pixel sums: fold over all 64 lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { v += __shfl_xor(v, o, 64); e += __shfl_xor(e, o, 64); }
    if (lane == 0) { wred[(wave * 8) * 38 + 36] = v; wred[(wave * 8) * 38 + 37] = e; }
  }
  __syncthreads();
  for (int i = tid; i < 8 * 36; i += NE_NTH) {
    const int g = i / 36, e = i % 36, k = e / 9, t = e % 9;
    float s = 0.f;
#pragma unroll
    for (int wv = 0; wv < NWAVE; ++wv) s += wred[(wv * 8 + g) * 38 + e];
    wpart[((size_t)slice * 9 + t) * 32 + g * 4 + k] = s;
  }
  if (tid == 0) {
    float bs = 0.f, es = 0.f;
#pragma unroll
    for (int wv = 0; wv < NWAVE; ++wv) { bs += wred[wv * 8 * 38 + 36]; es += wred[wv * 8 * 38 + 37]; }
    bpart[slice] = bs;
    bce_part[slice] = es;
  }
}


// ------------------------------------------------------------------ MFMA form (round 6)
// The same outputs with the three 288-MAC-per-pixel contractions on v_mfma_f32_16x16x32_f16
// (split-fp16 pieces, products a0b0 + a0b1 + a1b0 as in the convs), leaving the VALU only the
// normalise / LeakyReLU / split, the sigmoid / BCE and the bookkeeping:
//   (1) tap planes U[q][t] = sum_c a[q][c] w[c][t] of each source row (M = 16 pixels, N = 16
//       taps of which 9 are live, K = 32 channels): a lane's A fragment is one pixel's 8
//       channels, exactly as it loads them;
//   (2) per own row q, with g1 taken at q - d_t:
//         G[c][t] = sum_q a[q][c] g1[q - d_t]            (the final conv's weight gradient)
//         P[c][t] = sum_q [a[q][c] > 0] g1[q - d_t]      (indicator: exact in fp16)
//       (M = 16 channels, N = 16 taps, K = 32 pixels, the a / indicator fragments read from a
//       per-wave pixel-major LDS image with ds_read_b64_tr_b16, the g1 fragments from three
//       column-shifted copies of the g1 row);
//   and the block's InstanceNorm-backward reduce follows from them by two identities: with
//   ga[q][c] = sum_t w[c][t] g1[q - d_t] (the final conv's input gradient) and a = lrelu(xhat),
//       s2[c] = sum_q ga m xhat = sum_q ga a           = sum_t w[c][t] G[c][t]
//       s1[c] = sum_q ga m      = sum_t w[c][t] (slope S[t] + (1 - slope) P[c][t]),
//   m = lrelu'(xhat) in {1, slope} and S[t] = sum_q g1[q - d_t] (channel-free, on the VALU).
// Every quantity is restricted to the band's own rows q, as in net_end_kernel, so the band
// partials sum to the image's.  g1 is scaled by 2^kg (|g1| <= |cr| = the loss gradient scale,
// known at launch) and the weights by 2^kw (their block-wide maximum) into fp16's range; both
// are undone exactly.
template <int W> constexpr int nm_urs() { return W + 12; }  // plane row: col c at c + 4 (bank spread)
template <int W> constexpr int nm_grs() { return W + 8; }   // g1 copy row (fp16): x at x + 4
template <int W> constexpr size_t nm_lds() {
  return (size_t)NE_RING * 9 * nm_urs<W>() * 4        // tap planes
         + (size_t)NE_RING * 6 * nm_grs<W>() * 2        // g1 rows: [slot][kw][piece][GRS] fp16
         + (size_t)(W / 32) * 3 * 32 * 96;              // per-wave a0 / a1 / indicator images
}
constexpr int NM_IMG = 32 * 96;   // one per-wave image: 32 pixel rows of 32 channels (64 B + 32 pad)

EV_DEVINL f16x8 nm_pack(const unsigned (&v)[4]) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(f16x8, u4{v[0], v[1], v[2], v[3]});
}
EV_DEVINL f16x8 nm_tr(const char* r0, const char* r1) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) s16x4* lds_s16x4_ptr;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(r0));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(r1));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(f16x8, v);
}
EV_DEVINL f32x4 nm_mfma(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Schedule: one barrier per source row.  Step i (source row q = r0 - 2 + i):
//   [ (1) of row q: a, its fp16 pieces (registers), tap planes of row q -> plane slot q & 3 ]
//   barrier
//   [ x_hat / g1 of row q - 1 (planes of rows q - 2 .. q) -> g1 slot (q - 1) & 3;
//     (2) of own row q - 3 (g1 rows q - 4 .. q - 2, written before the barrier of step i - 1 or
//     earlier; its a fragments from the wave's image, written a step ago), then the image <- row
//     q - 2 ]
// Hazards: (1) of step i + 1 writes plane slot (q + 1) & 3 = (q - 3) & 3, which no wave reads
// after the barrier of step i; the g1 slot written at step i + 1, q & 3 = (q - 4) & 3, was last
// read by (2) of step i, before step i + 1's barrier.
template <int W, int TH>
__global__ __launch_bounds__(2 * W, W == 128 ? 2 : 1) void net_end_mfma_kernel(
    const float* __restrict__ y, const float2* __restrict__ st, const float* __restrict__ w14,
    const float* __restrict__ b14, const float* __restrict__ xt, const float* __restrict__ g_loss,
    float gscale, float* __restrict__ x_hat, float* __restrict__ g1out, float* __restrict__ bce_part,
    double2* __restrict__ part, float* __restrict__ wpart, float* __restrict__ bpart, int H) {
  constexpr int C = NE_C, NWAVE = W / 32, NTH = 64 * NWAVE;
  constexpr int URS = nm_urs<W>(), UROWS = 9 * URS, GRS = nm_grs<W>();
  extern __shared__ __attribute__((aligned(16))) float ne_sm[];
  float* uring = ne_sm;                                                   // [4][9][URS]
  _Float16* gring = reinterpret_cast<_Float16*>(ne_sm + NE_RING * UROWS);  // [4][3][2][GRS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, gq = lane >> 4;
  char* img = reinterpret_cast<char*>(gring + NE_RING * 6 * GRS) + wave * 3 * NM_IMG;
  const int tile = blockIdx.x, b = blockIdx.y, T = gridDim.x;
  const int r0 = tile * TH;
  const size_t HW = (size_t)H * W;
  const int px_w = wave * 32;   // the wave's 32 pixel columns

  // normalisation of this lane's 8 channels 8 gq .. 8 gq + 7, as channel pairs (net_end_kernel's)
  pkf2 fsr[4], fsb[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float2 f0 = norm_fs(st[(size_t)b * C + 8 * gq + 2 * k]);
    const float2 f1 = norm_fs(st[(size_t)b * C + 8 * gq + 2 * k + 1]);
    fsr[k] = pk2(f0.x, f1.x);
    fsb[k] = pk2(f0.y, f1.y);
  }
  // (1)'s B fragment: w14[c = 8 gq + j][t = l16] (t >= 9: 0), scaled by 2^kw, two fp16 pieces
  f16x8 wb0, wb1;
  int kw_;
  {
    float wv[8], m = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      wv[j] = l16 < 9 ? w14[(8 * gq + j) * 9 + l16] : 0.f;
      m = fmaxf(m, fabsf(wv[j]));
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    kw_ = f16_shift_of(m);
    const float s = ldexpf(1.f, kw_);
    unsigned h[4], lo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) split_f16x2_scaled(wv[2 * p], wv[2 * p + 1], s, h[p], lo[p]);
    wb0 = nm_pack(h);
    wb1 = nm_pack(lo);
  }
  const float uscale = ldexpf(1.f, -kw_);
  const float bias = b14 ? b14[0] : 0.f;
  const float cr = gscale * (g_loss ? *g_loss : 1.f);   // g_loss * scale / (B * P)
  const int kg = f16_shift_of(fabsf(cr));               // |g1| <= |cr|
  const float gsc = ldexpf(1.f, kg);

  // zero columns of the tap planes (col -1 and W), the two never-written g1 copy entries, and
  // the image (row r0 - 3 has no own-row (2); a defined image keeps the first pass finite)
  for (int i = tid; i < NE_RING * 9 * 2; i += NTH) {
    const int rw = i >> 1;
    uring[rw * URS + ((i & 1) ? W + 4 : 3)] = 0.f;
  }
  if (tid < NE_RING * 2 * 2) {   // [slot][piece][copy 0 at x = W-1 | copy 2 at x = 0] (x at x + 4)
    const int sl = tid >> 2, pc = (tid >> 1) & 1, which = tid & 1;
    gring[((sl * 3 + (which ? 2 : 0)) * 2 + pc) * GRS + (which ? 4 : W + 3)] = (_Float16)0.f;
  }

  const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + (size_t)b * HW * C), 0,
                                                    (int)(HW * C * 4), 0x00020000);
  auto load_row = [&](int q, float4 (&d)[2][2]) EV_LAMBDA_INLINE {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        d[g][h] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  ry, ((q * W + px_w + g * 16 + l16) * C + 8 * gq + 4 * h) * 4, 0, 0));
  };
  const bool xlane = lane < 32;   // the lanes that run the per-pixel part (pixel px_w + lane)
  auto load_tgt = [&](int r, float& d) EV_LAMBDA_INLINE {
    d = (r >= 0 && r < H && xlane) ? xt[(size_t)b * HW + (size_t)r * W + px_w + lane] : 0.f;
  };
  auto put_image = [&](const f16x8 (&pr)[3][2]) EV_LAMBDA_INLINE {
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
      for (int g = 0; g < 2; ++g)
        *reinterpret_cast<f16x8*>(img + t3 * NM_IMG + (g * 16 + l16) * 96 + 16 * gq) = pr[t3][g];
  };

  // G / P / S over the band's rows: the running sums of NE_FOLD rows at a time (G, P, S) are
  // folded into a second set (G2, P2, S2), so no fp32 sum runs over more rows than the 32-row
  // bands' did (64 rows in one accumulator took the saturated fixture's zero-bias residue of
  // decoder.13 from inside its gate to 22.8 x 2^-24 A)
  f32x4 G[2], P[2], G2[2], P2[2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) G[mb] = P[mb] = G2[mb] = P2[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float S[9], S2[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) S[t] = S2[t] = 0.f;
  float bsum = 0.f, bce = 0.f;
  // a0 / a1 / indicator fragments of source rows q - 1 (pa) and q - 2 (pb)
  // three register sets in rotation (step i: row q in R[i % 3], q - 1 in R[(i - 1) % 3], q - 2
  // in R[(i - 2) % 3]); the loop is unrolled by 6 so the rotation is a renaming, not copies
  f16x8 R0[3][2], R1[3][2], R2[3][2];
#pragma unroll
  for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
    for (int g = 0; g < 2; ++g) R0[t3][g] = R1[t3][g] = R2[t3][g] = f16x8{};
  put_image(R2);
  float4 ybuf[2][2][2];
  float tbuf[2];
  load_row(r0 - 2, ybuf[0]);
  load_row(r0 - 1, ybuf[1]);
  // the target of row q - 1 is read at step i: tbuf[i & 1] holds row r0 - 3 + i
  load_tgt(r0 - 3, tbuf[0]);
  load_tgt(r0 - 2, tbuf[1]);
  // (2)'s g1 fragment geometry: tap t = l16 (t >= 9: zero), 4 + 4 pixels of the wave's 32
  const int tkh = l16 < 9 ? l16 / 3 : 0, tkw = l16 < 9 ? l16 % 3 : 0;
  const bool tlive = l16 < 9;
  const int p4 = l16 & 3, qr = l16 >> 2;
  const int px0 = 4 * gq + qr, px1 = px0 + 16;
  // S[t]: column w feeds tap column kw = 0 unless w == 0, kw = 2 unless w == W - 1
  const float ml = (px_w + lane) != 0 ? 1.f : 0.f, mr = (px_w + lane) != W - 1 ? 1.f : 0.f;
  __syncthreads();

  auto step = [&](int i, float4 (&ycur)[2][2], float& tcur, f16x8 (&pn)[3][2], const f16x8 (&pb)[3][2])
                  EV_LAMBDA_INLINE {
    const int q = r0 - 2 + i;
    // ---- (1) a of source row q: registers (pn), tap planes into ring slot q & 3
    if (i < TH + 4 && q >= 0 && q < H) {   // block-uniform
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        float a[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 v = ycur[g][h];
          const pkf2 u0 = pkfma(pk2(v.x, v.y), fsr[2 * h], fsb[2 * h]);
          const pkf2 u1 = pkfma(pk2(v.z, v.w), fsr[2 * h + 1], fsb[2 * h + 1]);
          const pkf2 k0 = u0 * pk2(kSlope, kSlope), k1 = u1 * pk2(kSlope, kSlope);
          a[4 * h + 0] = fmaxf(u0.x, k0.x); a[4 * h + 1] = fmaxf(u0.y, k0.y);
          a[4 * h + 2] = fmaxf(u1.x, k1.x); a[4 * h + 3] = fmaxf(u1.y, k1.y);
        }
        unsigned h0[4], h1[4], ind[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          split_f16x2(a[2 * p], a[2 * p + 1], h0[p], h1[p]);
          ind[p] = (a[2 * p] > 0.f ? 0x3C00u : 0u) | (a[2 * p + 1] > 0.f ? 0x3C000000u : 0u);
        }
        pn[0][g] = nm_pack(h0);
        pn[1][g] = nm_pack(h1);
        pn[2][g] = nm_pack(ind);
      }
    } else {
#pragma unroll
      for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
        for (int g = 0; g < 2; ++g) pn[t3][g] = f16x8{};
    }
    load_row(q + 2, ycur);   // prefetch into the registers just consumed
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      f32x4 u = f32x4{0.f, 0.f, 0.f, 0.f};
      u = nm_mfma(pn[1][g], wb0, u);
      u = nm_mfma(pn[0][g], wb1, u);
      u = nm_mfma(pn[0][g], wb0, u);
      if (tlive)   // C/D: rows (pixels) 4 gq .. 4 gq + 3 of the group, column l16 = tap
        *reinterpret_cast<float4*>(uring + (q & 3) * UROWS + l16 * URS + 4 + px_w + g * 16 + 4 * gq) =
            make_float4(u[0] * uscale, u[1] * uscale, u[2] * uscale, u[3] * uscale);
    }
    __syncthreads();
    // ---- x_hat, g1 and BCE of row r = q - 1 from the planes of rows q - 2 .. q
    if (i >= 2 && i < TH + 4) {
      const int r = q - 1;
      const bool inrow = r >= 0 && r < H, own = r >= r0 && r < r0 + TH;
      if (xlane) {
        const int w = px_w + lane;
        float xh = 0.f;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const float* u = uring + ((q - 2 + kh) & 3) * UROWS + 4 + w - 1;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) xh += u[(kh * 3 + kw) * URS + kw];
        }
        xh += bias;
        float g = 0.f;
        if (inrow) {
          const float e = expf(-fabsf(xh));
          g = cr * (ne_sigmoid_e(xh, e) - tcur);
          if (own) {
            x_hat[(size_t)b * HW + (size_t)r * W + w] = xh;
            g1out[(size_t)b * HW + (size_t)r * W + w] = g;
            bce += ne_bce_e(xh, tcur, e);
            bsum += g;
          }
        }
        // S[t] = sum over own rows c of g1[c - d_t]: row r feeds tap row kh when
        // r in [r0 + 1 - kh, r0 + TH + 1 - kh), column w feeds kw unless the shifted
        // column falls outside the image (w = 0 for kw = 0, w = W - 1 for kw = 2)
#if EV_NE_BRFREE
        const float gl = g * ml, gr_ = g * mr;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
          if (r >= r0 + 1 - kh && r < r0 + TH + 1 - kh) {   // block-uniform
            S[3 * kh + 1] += g;
            S[3 * kh] += gl;
            S[3 * kh + 2] += gr_;
          }
#else
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
          if (r >= r0 + 1 - kh && r < r0 + TH + 1 - kh) {
            S[3 * kh + 1] += g;
            if (w != 0) S[3 * kh] += g;
            if (w != W - 1) S[3 * kh + 2] += g;
          }
#endif
        // g1 * 2^kg as two fp16 pieces into the three column-shifted copies of slot r & 3:
        // copy kw holds g1[x + 1 - kw] at x, stored at x + 4 (8-byte aligned fragment reads): the
        // writes to x = -1 and x = W land in pad entries no fragment reads, so they need no test
        const float gs = g * gsc;
        const _Float16 q0 = (_Float16)gs;
        const _Float16 q1 = (_Float16)(gs - (float)q0);
        _Float16* gr = gring + (size_t)(r & 3) * 6 * GRS + w + 3;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
#if !EV_NE_BRFREE
          const int x = w - 1 + kw;
          if (x >= 0 && x < W)
#endif
          {
            gr[(kw * 2 + 0) * GRS + kw] = q0;
            gr[(kw * 2 + 1) * GRS + kw] = q1;
          }
        }
      }
    }
    load_tgt(q + 1, tcur);   // row q + 1 is x_hat'd at step i + 2 (slot (i + 2) & 1)
    // ---- (2) G and P of own row c = q - 3 (its fragments in the wave's image)
    if (i >= 5 && i < TH + 5) {   // c in [r0, r0 + TH)
      const int c = q - 3;
      const _Float16* gr = gring + (size_t)((c - tkh + 1) & 3) * 6 * GRS + px_w + 4 * gq + 4;
      typedef short s16x4 __attribute__((ext_vector_type(4)));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      f16x8 gb[2];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const _Float16* gp = gr + (tkw * 2 + pc) * GRS;
        const s16x4 lo = *reinterpret_cast<const s16x4*>(gp);
        const s16x4 hi = *reinterpret_cast<const s16x4*>(gp + 16);
        // (tap columns t >= 9 of G / P are never read: their lanes' clamped reads need no zeroing)
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        gb[pc] = __builtin_bit_cast(f16x8, v);
      }
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        const int col = (16 * mb + 4 * p4) * 2;
        const f16x8 a0 = nm_tr(img + px0 * 96 + col, img + px1 * 96 + col);
        const f16x8 a1 = nm_tr(img + NM_IMG + px0 * 96 + col, img + NM_IMG + px1 * 96 + col);
        const f16x8 ai = nm_tr(img + 2 * NM_IMG + px0 * 96 + col, img + 2 * NM_IMG + px1 * 96 + col);
        G[mb] = nm_mfma(a1, gb[0], G[mb]);
        G[mb] = nm_mfma(a0, gb[1], G[mb]);
        G[mb] = nm_mfma(a0, gb[0], G[mb]);
        P[mb] = nm_mfma(ai, gb[1], P[mb]);
        P[mb] = nm_mfma(ai, gb[0], P[mb]);
      }
      if constexpr (TH > NE_FOLD) {
        if (((i - 5) & (NE_FOLD - 1)) == NE_FOLD - 1) {   // block-uniform
#pragma unroll
          for (int mb = 0; mb < 2; ++mb) {
            G2[mb] += G[mb];
            P2[mb] += P[mb];
            G[mb] = P[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int t = 0; t < 9; ++t) { S2[t] += S[t]; S[t] = 0.f; }
        }
      }
    }
    // the image now takes row q - 2, (2)'s row at step i + 1 (this wave's own LDS region: its
    // reads above were issued first and a wave's LDS operations complete in order)
    __builtin_amdgcn_sched_barrier(0);
    put_image(pb);
  };
  constexpr int NS = TH + 6, NM = NS - NS % 6;   // steps; those of the six-step loop
#if !EV_NE_UNROLL6
  auto rot = [&]() EV_LAMBDA_INLINE {
#pragma unroll
    for (int t3 = 0; t3 < 3; ++t3)
#pragma unroll
      for (int g = 0; g < 2; ++g) { R2[t3][g] = R1[t3][g]; R1[t3][g] = R0[t3][g]; }
  };
  (void)R2;
  static_assert(NS % 2 == 0, "two-step loop");
#pragma unroll 1
  for (int i = 0; i < NS; i += 2) {
    step(i, ybuf[0], tbuf[0], R0, R2);
    rot();
    step(i + 1, ybuf[1], tbuf[1], R0, R2);
    rot();
  }
#else
#pragma unroll 1
  for (int i = 0; i < NM; i += 6) {
    step(i, ybuf[0], tbuf[0], R0, R1);
    step(i + 1, ybuf[1], tbuf[1], R1, R2);
    step(i + 2, ybuf[0], tbuf[0], R2, R0);
    step(i + 3, ybuf[1], tbuf[1], R0, R1);
    step(i + 4, ybuf[0], tbuf[0], R1, R2);
    step(i + 5, ybuf[1], tbuf[1], R2, R0);
  }
  if constexpr (NS % 6 > 0) step(NM, ybuf[0], tbuf[0], R0, R1);
  if constexpr (NS % 6 > 1) step(NM + 1, ybuf[1], tbuf[1], R1, R2);
  if constexpr (NS % 6 > 2) step(NM + 2, ybuf[0], tbuf[0], R2, R0);
  if constexpr (NS % 6 > 3) step(NM + 3, ybuf[1], tbuf[1], R0, R1);
  if constexpr (NS % 6 > 4) step(NM + 4, ybuf[0], tbuf[0], R1, R2);
#endif
  __syncthreads();
  // ---- band partials, fixed order
  // G / P: C/D of wave w, M block mb: channel 16 mb + 4 gq + k (k = 0..3), tap l16
  float* red = ne_sm;   // [NWAVE][2 (G, P)][32 c][16 t]
  if (tlive) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = 16 * mb + 4 * gq + k;
        red[((wave * 2 + 0) * 32 + c) * 16 + l16] = G2[mb][k] + G[mb][k];
        red[((wave * 2 + 1) * 32 + c) * 16 + l16] = P2[mb][k] + P[mb][k];
      }
  }
  // S, bsum, bce: the 32 pixel lanes by a shuffle tree, then the waves
  float* sred = ne_sm + NWAVE * 2 * 32 * 16;   // [NWAVE][12]
  {
    float v[11];
#pragma unroll
    for (int t = 0; t < 9; ++t) v[t] = S2[t] + S[t];
    v[9] = bsum;
    v[10] = bce;
#pragma unroll
    for (int e = 0; e < 11; ++e) {
      float x = xlane ? v[e] : 0.f;
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) x += __shfl_xor(x, o, 64);
      if (lane == 0) sred[wave * 12 + e] = x;
    }
  }
  __syncthreads();
  const int slice = b * T + tile;
  if (tid < C) {   // channel c = tid
    const int c = tid;
    double Sd[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float s = 0.f;
#pragma unroll
      for (int wv = 0; wv < NWAVE; ++wv) s += sred[wv * 12 + t];
      Sd[t] = (double)s;
    }
    const double ig = 1.0 / (double)gsc;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float gt = 0.f, pt = 0.f;
#pragma unroll
      for (int wv = 0; wv < NWAVE; ++wv) {
        gt += red[((wv * 2 + 0) * 32 + c) * 16 + t];
        pt += red[((wv * 2 + 1) * 32 + c) * 16 + t];
      }
      const float gw = (float)((double)gt * ig);
      wpart[((size_t)slice * 9 + t) * 32 + c] = gw;
      const double wct = (double)w14[c * 9 + t];
      s2 += wct * (double)gw;
      s1 += wct * ((double)kSlope * Sd[t] + (1.0 - (double)kSlope) * (double)pt * ig);
    }
    part[(size_t)slice * C + c] = make_double2(s1, s2);
  }
  if (tid == 0) {
    float bs = 0.f, es = 0.f;
#pragma unroll
    for (int wv = 0; wv < NWAVE; ++wv) { bs += sred[wv * 12 + 9]; es += sred[wv * 12 + 10]; }
    bpart[slice] = bs;
    bce_part[slice] = es;
  }
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_net_end_tiles(int H, int W) {
  return ((W == 128 || W == 256) && ev_dim_ok(H) && H % NE_TH_MIN == 0) ? H / ne_th(H) : -1;
}

template <int W, int TH, bool MF>
static void net_end_launch(dim3 grid, hipStream_t st, const float* y13, const float* st13,
                           const float* w14, const float* b14, const float* x, const float* g_loss,
                           float gscale, float* x_hat, float* g1, float* bce_part, double* part,
                           float* wpart, float* bpart, int H) {
  auto k = MF ? net_end_mfma_kernel<W, TH> : net_end_kernel<W, TH>;
  constexpr size_t lds = MF ? nm_lds<W>() : ne_lds_u<W>();
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    once = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(ne_nth<W>()), lds, st, y13,
                     (const float2*)st13, w14, b14, x, g_loss, gscale, x_hat, g1, bce_part,
                     (double2*)part, wpart, bpart, H);
}

template <bool MF>
static int net_end_entry(const float* y13, const float* st13, const float* w14, const float* b14,
                         const float* x, const float* g_loss, float scale, float* x_hat,
                         float* g1, float* bce_part, double* part, float* wpart, float* bpart,
                         int B, int H, int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(y13 && st13 && w14 && x && x_hat && g1 && bce_part && part && wpart && bpart && B > 0,
             "net_end: null pointer");
  EV_REQUIRE(C == NE_C && ebsdvae_net_end_tiles(H, W) > 0,
             "net_end: C=%d %dx%d unsupported (C 32, W 128 or 256, H a multiple of %d)", C, H, W, NE_TH_MIN);
  const int T = ebsdvae_net_end_tiles(H, W);
  const float gscale = scale / ((float)B * (float)(H * W));
  const bool big = ne_th(H) == NE_TH;
#define EV_NE_LAUNCH(WW, TT)                                                                            \
  net_end_launch<WW, TT, MF>(dim3(T, B), (hipStream_t)stream, y13, st13, w14, b14, x, g_loss, gscale, \
                             x_hat, g1, bce_part, part, wpart, bpart, H)
  if (W == 128) {
    if (big) EV_NE_LAUNCH(128, NE_TH); else EV_NE_LAUNCH(128, NE_TH_MIN);
  } else {
    if (big) EV_NE_LAUNCH(256, NE_TH); else EV_NE_LAUNCH(256, NE_TH_MIN);
  }
#undef EV_NE_LAUNCH
  return evh::check_launch("net_end");
}

// the MFMA form (default) and the round-5 VALU form (A/B, EBSDVAE_NET_END_MFMA=0 in the engine)
extern "C" int ebsdvae_net_end(const float* y13, const float* st13, const float* w14, const float* b14,
                               const float* x, const float* g_loss, float scale, float* x_hat,
                               float* g1, float* bce_part, double* part, float* wpart, float* bpart,
                               int B, int H, int W, int C, ebsdvae_stream_t stream) {
  return net_end_entry<true>(y13, st13, w14, b14, x, g_loss, scale, x_hat, g1, bce_part, part, wpart,
                             bpart, B, H, W, C, stream);
}
extern "C" int ebsdvae_net_end_valu(const float* y13, const float* st13, const float* w14,
                                    const float* b14, const float* x, const float* g_loss, float scale,
                                    float* x_hat, float* g1, float* bce_part, double* part, float* wpart,
                                    float* bpart, int B, int H, int W, int C, ebsdvae_stream_t stream) {
  return net_end_entry<false>(y13, st13, w14, b14, x, g_loss, scale, x_hat, g1, bce_part, part, wpart,
                              bpart, B, H, W, C, stream);
}
