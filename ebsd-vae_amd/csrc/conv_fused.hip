// Fused input gradient + weight gradient of a 32 -> 32 channel 3x3 conv block (round 5): ONE
// pass over the block's output gradient gy and the previous block's pre-norm output y_prev
// computes both contractions of the backward of latice/model.py:95-97 / :102-106 (the
// full-resolution 32-channel layers encoder.1 and decoder.13 of VariationalAutoEncoderRawData):
//
//   input gradient   g[p][ci] = sum_{tap, co} gy[p + d(tap)][co] * Wd[tap][co][ci]   (Wd: the
//                    layer's input-gradient weight pack, ebsdvae_pack_conv_weights_split
//                    for_dgrad), with the previous block's InstanceNorm-backward reduce fused:
//                    the kernel writes h = g * lrelu'(xhat_prev) and the sums h, h * xhat_prev
//                    per 64-pixel slot (exactly conv3x3_pipe_kernel's fused reduce, P_ID), or,
//                    for an upsampled source (decoder.13), the 2x2 window sums of g (the
//                    upsample adjoint, FP_UPSUM) reduced once per window at H/2 x W/2;
//   weight gradient  dW[co][ci][tap] = sum_p gy[p][co] * act[p + d(tap)][ci], act =
//                    lrelu(IN(y_prev)) [upsampled], and db[co] = sum_p gy[p][co], as slice
//                    partials for the batched fixed-order reduce (wgrad_pipe_kernel's layout).
//
// The two kernels it replaces each read gy and y_prev from HBM and split gy into fp16 pieces
// (the input-gradient conv for its halo, the weight gradient for its tile): here both are read
// and staged once, and the y_prev values the reduce needs are the interior of the activation
// halo the weight gradient stages anyway.  At B = 256, 128 x 128 that is 1.07 GB (encoder.1)
// and 0.67 GB (decoder.13) less HBM traffic per step.
//
// Tiles are 8 x 8 pixels of one image; a block owns a slice (a contiguous run of tiles, row-major
// in the image, so consecutive tiles share halo columns in L2) and all 32 x 32 channels.  Per
// tile the block stages the 10 x 10 halo of gy and of the activation into LDS as fp16 pieces
// (pixel-major records, 96-B rows), double-buffered: four staging waves transform, split and
// write tile t+1 while their registers refill with tile t+2's loads, beside eight MFMA waves on
// tile t (one barrier per tile; DW_NOSPEC: the round-5 first form, where the MFMA waves stage
// between their taps).  MFMA waves:
//   weight gradient: wave w owns the (co 16 x ci 16) block (w & 1, (w >> 1) & 1) for the tile's
//     pixels 32 (w >> 2) .. +31 (one k-step of v_mfma_f32_16x16x32_f16 per tap; the two pixel
//     halves are folded at the end), operands by transposed LDS reads (ds_read_b64_tr_b16);
//   input gradient: wave w owns output pixels 16 (w & 3) .. +15 x ci 16 (w >> 2): per tap one
//     K = 32 (all gy channels) MFMA, A = the gy halo shifted by the tap (ds_read_b128), B = the
//     weight pack (resident in LDS; DW_NOSPEC: in registers).
// Each tap's LDS operands are read during the previous tap's MFMAs (one tap ahead).
// Both run the split-fp16 products a1 b0 + a0 b1 + a0 b0 (f16x3).  The gy operand carries one
// power-of-two scale per slice (from the applies' per-tile maxima, as the weight gradient's), the
// weights the pack's layer shift; the epilogue multiplies by the exact inverse.
#include <utility>

#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

constexpr int DW_C = 32;          // channels (cin == cout)
constexpr int DW_TS = 8;          // tile side
constexpr int DW_HP = 10;         // halo side
constexpr int DW_HALO = 100;      // halo pixels
constexpr int DW_RS = 96;         // LDS row stride of an image (32 ch x 2 B + 32 B pad)
constexpr int DW_PIECE = DW_HALO * DW_RS;          // one fp16 piece image
constexpr int DW_IMG = 2 * DW_PIECE;               // two pieces
constexpr int DW_BUF = 2 * DW_IMG;                 // gy image + activation image
constexpr int DW_WPACK = 4 * 10 * 2 * DW_C * 8 * 2;  // the dgrad pack (4 chunks x 10 taps x 2 pieces)
constexpr int DW_NTH = 512;       // the MFMA waves
constexpr int DW_NTH_SPEC = 768;  // SPEC: + 4 staging waves
constexpr int DW_ITEMS = DW_HALO * (DW_C / 4);     // float4 items of one halo tensor
constexpr size_t DW_LDS = (size_t)DW_WPACK + 2 * (size_t)DW_BUF + 4096;

typedef short dw_s16x4 __attribute__((ext_vector_type(4)));
typedef short dw_s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) dw_s16x4* dw_lds_s16x4_ptr;
typedef float dw_f32x4 __attribute__((ext_vector_type(4)));

// 8 halves of a k-major operand from two 4-row transposed reads (wgrad_pipe_kernel's tr_frag)
EV_DEVINL f16x8 dw_tr_frag(const char* r0, const char* r1) {
  const dw_s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((dw_lds_s16x4_ptr)(r0));
  const dw_s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((dw_lds_s16x4_ptr)(r1));
  const dw_s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(f16x8, v);
}
EV_DEVINL f16x8 dw_frag(const char* p) { return *reinterpret_cast<const f16x8*>(p); }
EV_DEVINL dw_f32x4 dw_mfma(f16x8 a, f16x8 b, dw_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
// 4 values -> their fp16 pieces at base (piece 0) and base + DW_PIECE (piece 1); s: the
// operand's power-of-two scale (1 for the activation)
EV_DEVINL void dw_store(char* base, float4 v, float s) {
  unsigned h01, l01, h23, l23;
  split_f16x2_scaled(v.x, v.y, s, h01, l01);
  split_f16x2_scaled(v.z, v.w, s, h23, l23);
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  *reinterpret_cast<u2*>(base) = u2{h01, h23};
  *reinterpret_cast<u2*>(base + DW_PIECE) = u2{l01, l23};
}

// compile-time loop (f(integral_constant<0>), ..., f(integral_constant<N-1>))
template <class F, int... I>
EV_DEVINL void dw_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>()), ...);
}
template <int N, class F>
EV_DEVINL void dw_for(F&& f) {
  dw_for_impl(f, std::make_integer_sequence<int, N>());
}

struct DwGeom {
  int ntx, lgx, lgp, tiles, tps, slices;
};

// UPS: the source is at H/2 x W/2 (decoder.13: ACT_NORM_UP, the input gradient summed over 2x2
// windows, FP_UPSUM); else the same resolution (encoder.1: ACT_NORM, P_ID)
// SPEC (round 5): 4 more waves (768 threads) do all the staging -- item loads, normalisation, fp16
// split, LDS stores, bias sums -- so the 8 MFMA waves run their taps without it and the staging
// VALU can issue beside their MFMAs on the same SIMDs; the input-gradient weights are then read
// from LDS per tap (the 168-VGPR budget of three waves per SIMD has no room for them)
template <bool UPS, bool SPEC>
__global__ __launch_bounds__(SPEC ? DW_NTH_SPEC : DW_NTH, 1) void dwgrad_fused_kernel(
    const float* __restrict__ gy, const float* __restrict__ gmax, int gmT,
    const char* __restrict__ wpack, const float* __restrict__ yprev, const float2* __restrict__ stp,
    float* __restrict__ hout, double2* __restrict__ ipart, float* __restrict__ wpart,
    float* __restrict__ bpart, int B, int H, int W, DwGeom g) {
  extern __shared__ __attribute__((aligned(16))) char dsm[];
  char* lw = dsm;                                  // resident dgrad weight pack
  char* lbuf = dsm + DW_WPACK;                     // two {gy image, act image} sets
  float* lred = reinterpret_cast<float*>(dsm + DW_WPACK + 2 * DW_BUF);   // 4 KiB scratch
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slice = blockIdx.x;
  const int t_beg = slice * g.tps, t_end = min(t_beg + g.tps, g.tiles);
  if (t_beg >= t_end) return;   // whole block, before any barrier
  const int Hs = UPS ? H / 2 : H, Ws = UPS ? W / 2 : W;
  const int per_img = g.ntx * g.ntx;
  constexpr int C = DW_C;
  constexpr int NTH = SPEC ? DW_NTH_SPEC : DW_NTH;   // threads
  constexpr int NST = SPEC ? NTH - DW_NTH : DW_NTH;  // staging threads
  constexpr int KS = (DW_ITEMS + NST - 1) / NST;     // items per staging thread per tensor
  const bool stager = SPEC && wave >= DW_NTH / 64;   // wave-uniform

  // ---- the dgrad weight pack -> LDS (resident), its layer shift from the trailer
  for (int i = tid; i < DW_WPACK / 16; i += NTH)
    reinterpret_cast<float4*>(lw)[i] = reinterpret_cast<const float4*>(wpack)[i];
  const int wshift = *reinterpret_cast<const int*>(wpack + DW_WPACK);
  // the slice's gy scale (its images' maxima), shared by both contractions
  const int gshift = f16_gshift(gmax, gmT, t_beg / per_img, (t_end - 1) / per_img);
  const float gsc = ldexpf(1.f, gshift);
  const float dsc = ldexpf(1.f, -(gshift + wshift));   // input-gradient undo
  const float wsc = 1.f / gsc;                          // weight-gradient undo

  // ---- item geometry (tile-invariant): item k of this thread is halo pixel hp = (tid + 512 k)
  // / 8 of the tile (row hr, column hc, -1 .. 8), channels 4 qd .. 4 qd + 3.  The same items
  // stage gy (this block's output gradient) and the activation source.
  const int sid = SPEC ? tid - DW_NTH : tid;   // staging thread index (SPEC: waves 8-11)
  const int qd = sid & 7;
  int hrc[KS], ldo[KS], gyo[KS], sro[KS];
  bool live[KS], inner[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    // pixel ranks with bits 0 / 1 swapped: each 16-lane group of a ds_write_b64 stores pixels
    // p, p + 2 (conflict-free, conv_wgrad.hip wg_store_perm)
    int hp = (sid + NST * k) >> 3;
    hp = (hp & ~3) | ((hp >> 1) & 1) | ((hp & 1) << 1);
    live[k] = hp < DW_HALO;
    const int hr = hp / DW_HP - 1, hc = hp % DW_HP - 1;
    hrc[k] = live[k] ? ((hr + 1) << 8) | (hc + 1) : 0;   // packed (row + 1, col + 1)
    inner[k] = live[k] && hr >= 0 && hr < DW_TS && hc >= 0 && hc < DW_TS;
    ldo[k] = hp * DW_RS + qd * 8;
    gyo[k] = ((hr * W + hc) * C + qd * 4) * 4;
    sro[k] = UPS ? (((hr >> 1) * Ws + (hc >> 1)) * C + qd * 4) * 4 : ((hr * W + hc) * C + qd * 4) * 4;
  }
  const int gimg = H * W * C * 4, simg = Hs * Ws * C * 4;

  // ---- tile coordinates: ntx is a power of two (host check)
  auto tile_at = [&](int t, int& b0, int& y0, int& x0) EV_LAMBDA_INLINE {
    const int rr = t & ((1 << g.lgp) - 1);
    b0 = t >> g.lgp;
    y0 = (rr >> g.lgx) * DW_TS;
    x0 = (rr & (g.ntx - 1)) * DW_TS;
  };
  // registers: gy and activation items of the loading tile (l*) and stats of the staging tile (s*)
  // two register slots (SPEC staging waves: tile u's loads are issued two tiles before it is
  // staged; the MFMA waves' in-tap staging uses slot 0 only)
  float4 rg[2][KS], ra[2][KS];
  float2 fl[2][4], fs[4];   // {rstd, -mean*rstd} of the item channels, loading / staging tile image
  int lb[2] = {0, 0}, ly[2] = {0, 0}, lx[2] = {0, 0}, sy = 0, sx = 0;
  auto issue = [&](int t, auto sl_c) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(sl_c)::value;
    tile_at(t, lb[sl], ly[sl], lx[sl]);
    const int lb_ = lb[sl], ly_ = ly[sl], lx_ = lx[sl];
    const auto rgy = __builtin_amdgcn_make_buffer_rsrc((void*)(gy + (size_t)lb_ * H * W * C), 0, gimg, 0x00020000);
    const auto rsr = __builtin_amdgcn_make_buffer_rsrc((void*)(yprev + (size_t)lb_ * Hs * Ws * C), 0, simg, 0x00020000);
    const int goff = (ly_ * W + lx_) * C * 4;
    const int soff = UPS ? ((ly_ >> 1) * Ws + (lx_ >> 1)) * C * 4 : goff;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      // rows above / below the image fall outside the descriptor range (read 0); the left /
      // right halo columns read a neighbouring row, zeroed at staging (dead items: out of range)
      const int o = live[k] ? goff + gyo[k] : (int)0x80000000;
      const int so = live[k] ? soff + sro[k] : (int)0x80000000;
      rg[sl][k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rgy, o, 0, 0));
      ra[sl][k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsr, so, 0, 0));
    }
    const float4* sp = reinterpret_cast<const float4*>(stp + (size_t)lb_ * C + qd * 4);
    const float4 u0 = sp[0], u1 = sp[1];
    fl[sl][0] = norm_fs(make_float2(u0.x, u0.y)); fl[sl][1] = norm_fs(make_float2(u0.z, u0.w));
    fl[sl][2] = norm_fs(make_float2(u1.x, u1.y)); fl[sl][3] = norm_fs(make_float2(u1.z, u1.w));
  };
  auto shift = [&](auto sl_c) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(sl_c)::value;
    sy = ly[sl]; sx = lx[sl];
#pragma unroll
    for (int i = 0; i < 4; ++i) fs[i] = fl[sl][i];
  };
  float4 tb = make_float4(0.f, 0.f, 0.f, 0.f);   // this thread's gy sums of the staging tile (bias)
  double bs[4] = {0.0, 0.0, 0.0, 0.0};
  // stage item k (gy and activation) of the staging tile into set buf
  auto stage = [&](int k, char* buf, auto sl_c) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(sl_c)::value;
    if (!live[k]) return;
    const int hr = (hrc[k] >> 8) - 1, hc = (hrc[k] & 255) - 1;
    const bool in = (unsigned)(sy + hr) < (unsigned)H && (unsigned)(sx + hc) < (unsigned)W;
    float4 v = in ? rg[sl][k] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (inner[k]) { tb.x += v.x; tb.y += v.y; tb.z += v.z; tb.w += v.w; }
    dw_store(buf + ldo[k], v, gsc);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (in) {
      const float4 r = ra[sl][k];
      a = make_float4(normact_fs(r.x, fs[0]), normact_fs(r.y, fs[1]), normact_fs(r.z, fs[2]),
                      normact_fs(r.w, fs[3]));
    }
    dw_store(buf + DW_IMG + ldo[k], a, 1.f);
  };

  // ---- per-lane MFMA geometry
  const int n16 = lane & 15, gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  // weight gradient: (co block, ci block, pixel half) of this wave
  const int wco = wave & 1, wci = (wave >> 1) & 1, wks = wave >> 2;
  const int px0 = 32 * wks + 4 * gq + q4, px1 = px0 + 16;
  const int hq0 = (px0 >> 3) * DW_HP + (px0 & 7), hq1 = (px1 >> 3) * DW_HP + (px1 & 7);   // halo index of (px - (1,1))
  const int acol = (wco * 16 + 4 * p4) * 2, bcol = (wci * 16 + 4 * p4) * 2;
  // input gradient: (pixel block, ci block) of this wave; lane = output pixel n16 of the block's
  // A rows, k-group gq = gy channels 8 gq .. 8 gq + 7
  const int dpx = (wave & 3) * 16, dci = (wave >> 2) * 16;
  const int apx = dpx + n16;                                  // A row pixel
  const int ahq = (apx >> 3) * DW_HP + (apx & 7);
  dw_f32x4 accw[9], accd;
#pragma unroll
  for (int t = 0; t < 9; ++t) accw[t] = dw_f32x4{0.f, 0.f, 0.f, 0.f};
  accd = dw_f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- epilogue of the input gradient for the tile at (b0, y0, x0): h and the fused reduce
  // (C layout: lane -> ci dci + n16, output pixels dpx + 4 gq + r).  Its y_prev values and
  // statistics are loaded at the start of the tile (pre_load), so their latency hides under
  // the tile's MFMAs; the per-slot sums go through a two-deep LDS ring and are combined by
  // threads 0-31 at the start of the next tile (after its barrier), so the epilogue itself
  // has no barrier.
  const int eci = dci + n16;
  const int T = (H / DW_TS) * (W / DW_TS);   // slots (8 x 8 tiles) per image
  double2* red = reinterpret_cast<double2*>(lred);   // [2 tiles][4 pixel-block waves][2 ci blocks][16]
  const int rr = (dpx + 4 * gq) >> 3, cc = (4 * gq) & 7;   // this lane's pixels: tile row rr, columns cc..
  float pv[4];
  float2 psp;
  auto pre_load = [&](int tt) EV_LAMBDA_INLINE {
    int b0, y0, x0;
    tile_at(tt, b0, y0, x0);
    psp = stp[(size_t)b0 * C + eci];
    if constexpr (!UPS) {
      const float* yp = yprev + (((size_t)b0 * H + y0 + rr) * W + x0 + cc) * C + eci;
#pragma unroll
      // default policy: the other ci block's wave reads the other half of each 128-B line
      // (non-temporal half-line loads fetched lines twice: -20 us with the default)
      for (int r = 0; r < 4; ++r) pv[r] = yp[r * C];
    } else {
      // lanes gq < 2 own the windows (wr, wc), (wr, wc + 1) at H/2 x W/2; the others load the
      // same addresses (no divergent branch, the values are unused)
      const int wr = (y0 >> 1) + (rr >> 1), wc = (x0 >> 1) + ((cc & 4) >> 1);
      const float* yp = yprev + (((size_t)b0 * (H >> 1) + wr) * (W >> 1) + wc) * C + eci;
      pv[0] = yp[0];
      pv[1] = yp[C];
      pv[2] = pv[3] = 0.f;
    }
  };
  auto combine = [&](int tt) EV_LAMBDA_INLINE {   // threads 0-31, the slot sums of tile tt
    int b0, y0, x0;
    tile_at(tt, b0, y0, x0);
    const int cb = tid >> 4, n = tid & 15;
    const double2* rb = red + ((tt - t_beg) & 1) * 128;
    double u = 0.0, w = 0.0;
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      const double2 e = rb[(pb * 2 + cb) * 16 + n];
      u += e.x; w += e.y;
    }
    const int slot = (y0 / DW_TS) * (W / DW_TS) + x0 / DW_TS;
    ipart[((size_t)b0 * T + slot) * C + tid] = make_double2(u, w);
  };
  auto epilogue = [&](int tt) EV_LAMBDA_INLINE {
    int b0, y0, x0;
    tile_at(tt, b0, y0, x0);
    const float2 sp = psp;
    const float spc = -sp.x * sp.y;
    float s1 = 0.f, s2 = 0.f;
    if constexpr (!UPS) {
      float* hp = hout + (((size_t)b0 * H + y0 + rr) * W + x0 + cc) * C + eci;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = accd[r] * dsc;
        const float y = pv[r];
        const float x = fmaf(y, sp.y, spc);
        const float ga = y > sp.x ? v : v * kSlope;
        s1 += ga;
        s2 = fmaf(ga, x, s2);
        hp[r * C] = ga;   // half lines: the L2 merges the two ci blocks' halves
      }
      s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64); s2 += __shfl_xor(s2, 32, 64);
    } else {
      // window sums: this lane's pixel pairs (cc, cc+1), (cc+2, cc+3) of tile row rr, and the
      // row below from lane + 32 (gq + 2: same columns, rr + 1); lanes gq < 2 own the windows
      const float v0 = accd[0] * dsc, v1 = accd[1] * dsc, v2 = accd[2] * dsc, v3 = accd[3] * dsc;
      const float t0 = v0 + v1, t1 = v2 + v3;
      const float b0s = __shfl_xor(t0, 32, 64), b1s = __shfl_xor(t1, 32, 64);
      if (gq < 2) {
        const int wr = (y0 >> 1) + (rr >> 1), wc = (x0 >> 1) + (cc >> 1);
        float* hp = hout + (((size_t)b0 * (H >> 1) + wr) * (W >> 1) + wc) * C + eci;
        const float gs[2] = {t0 + b0s, t1 + b1s};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float y = pv[j];
          const float x = fmaf(y, sp.y, spc);
          const float ga = y > sp.x ? gs[j] : gs[j] * kSlope;
          s1 += ga;
          s2 = fmaf(ga, x, s2);
          hp[j * C] = ga;
        }
      }
      s1 += __shfl_xor(s1, 16, 64); s2 += __shfl_xor(s2, 16, 64);
    }
    // the 4 pixel-block waves of a ci block -> one slot sum per channel, fixed order (combine)
    if (gq == 0)
      red[((tt - t_beg) & 1) * 128 + ((wave & 3) * 2 + (wave >> 2)) * 16 + n16] =
          make_double2((double)s1, (double)s2);
  };

  // ---- prologue: tile t_beg staged into set 0, tile t_beg + 1 (clamped) in the registers
  const std::integral_constant<int, 0> S0;
  const std::integral_constant<int, 1> S1;
  if (stager) {             // SPEC: tiles t_beg, t_beg + 1 into slots 0, 1
    issue(t_beg, S0);
    issue(min(t_beg + 1, t_end - 1), S1);
  } else if (!SPEC) {
    issue(t_beg, S0);
    shift(S0);
  }
  __syncthreads();   // the weight pack is in LDS before anyone reads it (and before set 0 is read)
  if (stager) {
    shift(S0);
#pragma unroll
    for (int k = 0; k < KS; ++k) stage(k, lbuf, S0);
    bs[0] += (double)tb.x; bs[1] += (double)tb.y; bs[2] += (double)tb.z; bs[3] += (double)tb.w;
    issue(min(t_beg + 2, t_end - 1), S0);
  } else if (!SPEC) {
#pragma unroll
    for (int k = 0; k < KS; ++k) stage(k, lbuf, S0);
    bs[0] += (double)tb.x; bs[1] += (double)tb.y; bs[2] += (double)tb.z; bs[3] += (double)tb.w;
    issue(min(t_beg + 1, t_end - 1), S0);
  }
  __syncthreads();

  // the input-gradient B fragments of this lane (the pack: 9 taps x 2 pieces) stay in registers
  // for the whole slice (72 VGPRs; read once instead of once per tile: -30 us at B = 256)
  f16x8 dbr[9][2];
  if constexpr (!SPEC) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int i = 0; i < 2; ++i) dbr[tap][i] = dw_frag(lw + ((((gq * 10 + tap) * 2 + i) * C) + eci) * 16);
  }
  if (stager) {
    // SPEC staging waves (their own loop, so their registers are not live beside the MFMA
    // waves' accumulators): tile t+1 into the other set, then its registers refill with t+2
    // tile t+1 is in slot (t + 1 - t_beg) & 1; its slot refills with tile t+3
    auto stager_tile = [&](int t, auto sl_c) EV_LAMBDA_INLINE {
      char* nbuf = lbuf + (1 - ((t - t_beg) & 1)) * DW_BUF;
      shift(sl_c);
      tb = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < KS; ++k) stage(k, nbuf, sl_c);
      issue(min(t + 3, t_end - 1), sl_c);
      const float keep = (t + 1 < t_end) ? 1.f : 0.f;
      bs[0] += (double)(tb.x * keep); bs[1] += (double)(tb.y * keep);
      bs[2] += (double)(tb.z * keep); bs[3] += (double)(tb.w * keep);
      __syncthreads();
    };
    for (int t = t_beg; t < t_end; t += 2) {
      stager_tile(t, S1);
      if (t + 1 < t_end) stager_tile(t + 1, S0);
    }
  } else {
  for (int t = t_beg; t < t_end; ++t) {
    const int cur = (t - t_beg) & 1;
    const char* gimgp = lbuf + cur * DW_BUF;
    const char* aimgp = gimgp + DW_IMG;
    char* nbuf = lbuf + (1 - cur) * DW_BUF;
    pre_load(t);
    if (t > t_beg && tid < C) combine(t - 1);   // the previous tile's slot sums (behind its barrier)
    if constexpr (!SPEC) {
      shift(S0);
      tb = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // weight-gradient A fragments (gy, k = this wave's 32 pixels): one read per piece
    f16x8 wa[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      wa[i] = dw_tr_frag(gimgp + i * DW_PIECE + (hq0 + 11) * DW_RS + acol,
                         gimgp + i * DW_PIECE + (hq1 + 11) * DW_RS + acol);
    // this tap's LDS operands were read one tap ahead (their latency under the previous tap's
    // MFMAs); the first tap's here
    f16x8 wbc[2], dac[2];
    auto ld_tap = [&](auto tap_c, f16x8* wbv, f16x8* dav) EV_LAMBDA_INLINE {
      constexpr int tap = decltype(tap_c)::value;
      constexpr int toff = (tap / 3) * DW_HP + tap % 3;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        wbv[i] = dw_tr_frag(aimgp + i * DW_PIECE + (hq0 + toff) * DW_RS + bcol,
                            aimgp + i * DW_PIECE + (hq1 + toff) * DW_RS + bcol);
        dav[i] = dw_frag(gimgp + i * DW_PIECE + (ahq + toff) * DW_RS + gq * 16);
      }
    };
    ld_tap(std::integral_constant<int, 0>(), wbc, dac);
    dw_for<9>([&](auto tap_c) EV_LAMBDA_INLINE {
      constexpr int tap = decltype(tap_c)::value;
      f16x8 wbn[2], dan[2];
      if constexpr (tap < 8) ld_tap(std::integral_constant<int, tap + 1>(), wbn, dan);
      __builtin_amdgcn_sched_barrier(0);   // issued ahead of this tap's MFMAs
      const f16x8* wb = wbc;
      const f16x8* da = dac;
      f16x8 dbt[2];
      if constexpr (SPEC) {
#pragma unroll
        for (int i = 0; i < 2; ++i) dbt[i] = dw_frag(lw + ((((gq * 10 + tap) * 2 + i) * C) + eci) * 16);
      }
      const f16x8* db = SPEC ? dbt : dbr[tap];
      accw[tap] = dw_mfma(wa[1], wb[0], accw[tap]);
      accw[tap] = dw_mfma(wa[0], wb[1], accw[tap]);
      accw[tap] = dw_mfma(wa[0], wb[0], accw[tap]);
      accd = dw_mfma(da[1], db[0], accd);
      accd = dw_mfma(da[0], db[1], accd);
      accd = dw_mfma(da[0], db[0], accd);
      // staging of tile t+1 between the taps (item k at tap 2 k + 1), then its register
      // refill is tile t+2's load (issued once, after the last item)
      if constexpr (!SPEC) {
        dw_for<KS>([&](auto k_c) EV_LAMBDA_INLINE {
          constexpr int k = decltype(k_c)::value;
          if constexpr (tap == 2 * k + 1) stage(k, nbuf, S0);
        });
        if constexpr (tap == 2 * KS) issue(min(t + 2, t_end - 1), S0);
      }
      if constexpr (tap < 8) {
#pragma unroll
        for (int i = 0; i < 2; ++i) { wbc[i] = wbn[i]; dac[i] = dan[i]; }
      }
    });
    // branch-free (the surplus copy of the last tile is weighted 0), and 24 wait states before
    // the epilogue reads accd: with a conditional block here, hipcc (ROCm 7.2) put the epilogue's
    // first VALU read of the last MFMA's result right behind the branch on the skipping path,
    // without the wait states an MFMA result needs (wrong input gradients on every slice's last
    // tile, tools/debug/dw_ups.py)
    if constexpr (!SPEC) {
      const float keep = (t + 1 < t_end) ? 1.f : 0.f;
      bs[0] += (double)(tb.x * keep); bs[1] += (double)(tb.y * keep);
      bs[2] += (double)(tb.z * keep); bs[3] += (double)(tb.w * keep);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    epilogue(t);
    accd = dw_f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
  }
  }
  if (tid < C) combine(t_end - 1);

  // ---- weight-gradient partials: fold the two pixel halves (waves 4-7 into 0-3) through LDS
  float* xs = reinterpret_cast<float*>(lbuf);   // LDS sets are free after the last barrier
  if (wks == 1) {   // waves 4-7 (SPEC staging waves: wks == 2)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) xs[((wave - 4) * 36 + t * 4 + r) * 64 + lane] = accw[t][r];
  }
  __syncthreads();
  if (wks == 0) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = accw[t][r] + xs[(wave * 36 + t * 4 + r) * 64 + lane];
        const int co = wco * 16 + gq * 4 + r, ci = wci * 16 + n16;
        __builtin_nontemporal_store(v * wsc, wpart + (((size_t)slice * 9 + t) * C + co) * C + ci);
      }
  }
  __syncthreads();
  // bias partial: threads with the same channel group qd fold their sums in a fixed order
  double* xb = reinterpret_cast<double*>(lbuf);
#pragma unroll
  for (int i = 0; i < 4; ++i) xb[i * NTH + tid] = bs[i];
  __syncthreads();
  if (tid < C) {
    const int qq = tid >> 2, i = tid & 3;
    double sum = 0.0;
    for (int m = qq; m < NTH; m += 8) sum += xb[i * NTH + m];
    bpart[(size_t)slice * C + tid] = (float)sum;
  }
}

// slices: one block per slice, ~one per CU (the block fills a CU: 8 waves, ~120 KB LDS)
static bool dw_geom(int B, int H, int W, DwGeom* g) {
  if (B <= 0 || H != W || H % DW_TS || (H / DW_TS) & (H / DW_TS - 1)) return false;
  if (!ev_buf_bytes_ok(4LL * H * W * DW_C)) return false;
  g->ntx = W / DW_TS;
  g->lgx = __builtin_ctz(g->ntx);
  g->lgp = 2 * g->lgx;
  g->tiles = B * g->ntx * g->ntx;
  int tps = 4;
  while ((g->tiles + tps - 1) / tps > 256) tps *= 2;
  g->tps = tps;
  g->slices = (g->tiles + tps - 1) / tps;
  return true;
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_conv3x3_dwgrad_slices(int B, int H, int W, int cin, int cout) {
  DwGeom g;
  if (cin != DW_C || cout != DW_C || !dw_geom(B, H, W, &g)) return -1;
  return g.slices;
}

extern "C" int ebsdvae_conv3x3_dwgrad_stat_tiles(int H, int W) {
  if (!ev_dim_ok(H) || !ev_dim_ok(W) || H % DW_TS || W % DW_TS) return -1;
  return (H / DW_TS) * (W / DW_TS);
}

extern "C" int ebsdvae_conv3x3_dwgrad_f16(const float* gy, const float* gmax, int gm_tiles,
                                          const void* wpack, const float* y_prev,
                                          const float* st_prev, int src_mode, float* gin,
                                          double* part, float* wpart, float* bpart, int B, int H,
                                          int W, int cin, int cout, ebsdvae_stream_t stream) {
  DwGeom g;
  EV_REQUIRE(gy && gmax && gm_tiles > 0 && wpack && y_prev && st_prev && gin && part && wpart && bpart && B > 0,
             "conv3x3_dwgrad_f16: null pointer, empty batch or no gradient maxima");
  EV_REQUIRE(src_mode == ACT_NORM || src_mode == ACT_NORM_UP,
             "conv3x3_dwgrad_f16: src_mode %d (ACT_NORM or ACT_NORM_UP)", src_mode);
  EV_REQUIRE(cin == DW_C && cout == DW_C && dw_geom(B, H, W, &g),
             "conv3x3_dwgrad_f16: unsupported shape B=%d H=%d W=%d cin=%d cout=%d", B, H, W, cin, cout);
  hipStream_t s = (hipStream_t)stream;
  auto launch = [&](auto kern, int nth) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DW_LDS);
    hipLaunchKernelGGL(kern, dim3(g.slices), dim3(nth), DW_LDS, s, gy, gmax, gm_tiles,
                       (const char*)wpack, y_prev, (const float2*)st_prev, gin, (double2*)part, wpart,
                       bpart, B, H, W, g);
  };
#ifdef DW_NOSPEC   // A/B: every wave stages between its taps (no staging waves)
  if (src_mode == ACT_NORM) launch(dwgrad_fused_kernel<false, false>, DW_NTH);
  else launch(dwgrad_fused_kernel<true, false>, DW_NTH);
#else
  if (src_mode == ACT_NORM) launch(dwgrad_fused_kernel<false, true>, DW_NTH_SPEC);
  else launch(dwgrad_fused_kernel<true, true>, DW_NTH_SPEC);
#endif
  return evh::check_launch("conv3x3_dwgrad_f16");
}
