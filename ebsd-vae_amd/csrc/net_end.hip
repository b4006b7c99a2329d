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
constexpr int NE_C = 32, NE_TH = 32;
constexpr int NE_RING = 4;                 // ring slots (a and g1): slot(row) = (row - r0 + k) & 3
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
template <int W>
__global__ __launch_bounds__(ne_nth<W>(), W == 128 ? 2 : 1) void net_end_kernel(
    const float* __restrict__ y, const float2* __restrict__ st, const float* __restrict__ w14,
    const float* __restrict__ b14, const float* __restrict__ xt, const float* __restrict__ g_loss,
    float gscale, float* __restrict__ x_hat, float* __restrict__ g1out, float* __restrict__ bce_part,
    double2* __restrict__ part, float* __restrict__ wpart, float* __restrict__ bpart, int H) {
  constexpr int C = NE_C, TH = NE_TH, WP = ne_wp<W>(), UROW = ne_urow<W>();
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

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_net_end_tiles(int H, int W) {
  return ((W == 128 || W == 256) && ev_dim_ok(H) && H % NE_TH == 0) ? H / NE_TH : -1;
}

template <int W>
static void net_end_launch(dim3 grid, hipStream_t st, const float* y13, const float* st13,
                           const float* w14, const float* b14, const float* x, const float* g_loss,
                           float gscale, float* x_hat, float* g1, float* bce_part, double* part,
                           float* wpart, float* bpart, int H) {
  auto k = net_end_kernel<W>;
  constexpr size_t lds = ne_lds_u<W>();
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    once = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(ne_nth<W>()), lds, st, y13,
                     (const float2*)st13, w14, b14, x, g_loss, gscale, x_hat, g1, bce_part,
                     (double2*)part, wpart, bpart, H);
}

extern "C" int ebsdvae_net_end(const float* y13, const float* st13, const float* w14, const float* b14,
                               const float* x, const float* g_loss, float scale, float* x_hat,
                               float* g1, float* bce_part, double* part, float* wpart, float* bpart,
                               int B, int H, int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(y13 && st13 && w14 && x && x_hat && g1 && bce_part && part && wpart && bpart && B > 0,
             "net_end: null pointer");
  EV_REQUIRE(C == NE_C && ebsdvae_net_end_tiles(H, W) > 0,
             "net_end: C=%d %dx%d unsupported (C 32, W 128 or 256, H a multiple of %d)", C, H, W, NE_TH);
  const int T = ebsdvae_net_end_tiles(H, W);
  const float gscale = scale / ((float)B * (float)(H * W));
  if (W == 128)
    net_end_launch<128>(dim3(T, B), (hipStream_t)stream, y13, st13, w14, b14, x, g_loss, gscale, x_hat,
                        g1, bce_part, part, wpart, bpart, H);
  else
    net_end_launch<256>(dim3(T, B), (hipStream_t)stream, y13, st13, w14, b14, x, g_loss, gscale, x_hat,
                        g1, bce_part, part, wpart, bpart, H);
  return evh::check_launch("net_end");
}
