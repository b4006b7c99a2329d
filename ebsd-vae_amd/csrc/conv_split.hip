// 3x3 stride-1 pad-1 convolution (forward and input gradient) on the bf16 MFMA with split
// operands: every fp32 operand x is carried as NP bf16 pieces
//     x0 = bf16(x), x1 = bf16(x - x0) [, x2 = bf16(x - x0 - x1)]
// (8 mantissa bits each; |x - sum| <= 2^-18 |x| for NP = 2, 2^-27 |x| for NP = 3), and each
// product keeps the terms of total order < NP (bf16 x bf16 products are exact in fp32,
// accumulation is fp32):
//   NP = 2 ("bf16x3"): a0b0 + a0b1 + a1b0                    3 MFMAs, ~2^-16.5 rel. error
//   NP = 3 ("bf16x6"): + a0b2 + a2b0 + a1b1                  6 MFMAs, ~2^-25 (fp32 grade)
// at 16x the fp32-MFMA rate per v_mfma_f32_32x32x16_bf16: 5.3x / 2.7x the fp32 MFMA peak
// (split-precision MFMA path, gated by the parity tests).  Replaces the same reference ops as conv_fwd.hip:
// nn.Conv2d / nn.ConvTranspose2d forward (latice/model.py:95,102-104) and their input
// gradients, with the same fused prologue (InstanceNorm + LeakyReLU [+ pool / upsample] of
// the producer's saved output) and epilogue (bias, InstanceNorm partials, optional fused
// InstanceNorm-backward reduce).
//
// GEMM view as in conv_fwd.hip: M = output pixels, N = Cout, K = 9 taps x Cin swept in
// 8-channel chunks.  One 32x32x16 k-step covers two taps: lane half h = lane >> 5 takes tap
// 2s + h (s = 0..4; a zero tenth tap pads the odd tap count).
//   LDS halo record per pixel (48 B): piece 0 [8 ch] | piece 1 [8 ch] | piece 2 or pad ->
//     one ds_read_b128 per piece, conflict-free over 16 consecutive pixels (3 x 16 B granules
//     apart);
//   LDS weight slab per chunk: [tap 0..9][piece][Cout][8 ch] bf16, DMA'd by global_load_lds
//     from the split pack (ebsdvae_pack_conv_weights_split).
#include "conv_common.h"
#include "instnorm_fin.h"

#include <stdlib.h>
#include <type_traits>

namespace ev {

static_assert(NP_F16 == EBSDVAE_PIECES_F16, "piece-format id");

#ifdef EV_PIPE_TRACE   // diagnostic build only: per-wave cycle split of conv3x3_pipe_kernel
__device__ unsigned long long ev_pipe_trace[4096 * 8 * 6];
#define EV_T(x) unsigned long long x = __builtin_amdgcn_s_memtime()
#define EV_TACC(acc, t0) acc += __builtin_amdgcn_s_memtime() - t0
#else
#define EV_T(x)
#define EV_TACC(acc, t0)
#endif


typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int XCK = 8;      // input channels per chunk
// Source mode of the pipelined kernel only (not an ActMode of the ABI): the input is the first
// block's activation lrelu(IN(y0)) with y0 = conv(x, w0) + b0 recomputed from the image x while
// the halo is staged (ebsdvae_conv3x3_fwd_split_first), so y0 is never read
constexpr int ACT_FIRST = 5;
constexpr int FIRST_WTAB = 8 * 10 * 4;   // [chunk * 2 + half][tap 0..8, bias][4 channels] floats
constexpr int XTAPS = 10;   // 9 taps + one zero tap
constexpr int XPS = 48;     // halo pixel record (bytes)
#ifndef EV_PIPE_EPI_G
#define EV_PIPE_EPI_G 8   // fused IN-backward loads in flight per batch, NF > 1 (VGPR budget)
#endif

// x -> NP bf16 pieces (the remainder is re-split exactly in fp32 at every step)
template <int NP>
EV_DEVINL void split_bf16(float x, __bf16 (&p)[NP]) {
  float r = x;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    p[i] = (__bf16)r;
    r -= (float)p[i];
  }
}

// Piece format NP_F16 ("f16x3"): two fp16 pieces
//     x0 = f16(x), x1 = f16(x - x0)      (11 significand bits each, |x - x0 - x1| <= 2^-23 |x|
//                                          for normal x1, 2^-25 absolute below it)
// and the three products a0b0 + a0b1 + a1b0 on v_mfma_f32_32x32x16_f16 (the dropped a1b1 is
// <= 2^-24 relative): ~2^-22.5 per product, at the bf16x3 rate.  fp16's range is narrow, so
// the weights of each layer are packed as w * 2^k, k from the layer's max |w| (max |w| 2^k in
// [2^11, 2^12): pack_wmax_kernel + pack_split_kernel, stored in the pack's trailer) and the
// epilogue multiplies the accumulators by the exact 2^-k.  Forward operands are normalised
// activations (IN + LeakyReLU, |x| <= sqrt(H*W - 1) by construction), which fp16 holds as
// they are; the gradient operand of input-gradient launches is scaled per image by a power of
// two from its per-tile maxima (GS), and so is the weight gradient's per slice
// (conv_wgrad.hip).

template <int NP>
EV_DEVINL void split4(float4 v, bf16x4 (&out)[npc(NP)]) {
  if constexpr (NP == NP_F16) {
    unsigned h01, l01, h23, l23;
    split_f16x2(v.x, v.y, h01, l01);
    split_f16x2(v.z, v.w, h23, l23);
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    out[0] = __builtin_bit_cast(bf16x4, u2{h01, h23});
    out[1] = __builtin_bit_cast(bf16x4, u2{l01, l23});
    return;
  }
  const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if constexpr (NP == NP_F16) {   // fp16 bit patterns in the 16-bit piece slots
      const _Float16 h0 = (_Float16)e[c];
      const _Float16 h1 = (_Float16)(e[c] - (float)h0);
      out[0][c] = __builtin_bit_cast(__bf16, h0);
      out[1][c] = __builtin_bit_cast(__bf16, h1);
    } else {
      __bf16 p[NP];
      split_bf16<NP>(e[c], p);
#pragma unroll
      for (int i = 0; i < NP; ++i) out[i][c] = p[i];
    }
  }
}

// one 32x32x16 product of two piece fragments (bf16, or fp16 bits for NP_F16)
// split4 of v * s (s a power of two) for the fp16 pieces: split_f16x2_scaled
EV_DEVINL void split4_f16_scaled(float4 v, float s, bf16x4 (&out)[2]) {
  unsigned h01, l01, h23, l23;
  split_f16x2_scaled(v.x, v.y, s, h01, l01);
  split_f16x2_scaled(v.z, v.w, s, h23, l23);
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  out[0] = __builtin_bit_cast(bf16x4, u2{h01, h23});
  out[1] = __builtin_bit_cast(bf16x4, u2{l01, l23});
}

template <int NP>
EV_DEVINL f32x16 mfma_piece(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (NP == NP_F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

EV_DEVINL bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

// 16-B buffer load (32-bit byte offset; out-of-range offsets read 0 without a memory access)
EV_DEVINL float4 bload4(__amdgpu_buffer_rsrc_t rs, int off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
}

template <int NP, int NWV, int WM, int MF, int NF, int KX, int MODE, int FP>
__global__ __launch_bounds__(NWV * 64, 2) void conv3x3_split_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, const char* __restrict__ wp,
    const float* __restrict__ bias, float* __restrict__ y, float2* __restrict__ spart,
    float* __restrict__ act_out, int B, int H, int W, int Cin, int TH,
    const float* __restrict__ yprev, const float2* __restrict__ stprev, double2* __restrict__ ipart) {
  constexpr int WN = NWV / WM;
  constexpr int NT = WN * NF * 32;               // == Cout
  constexpr int MW = MF * 32;
  constexpr int NTHR = NWV * 64;
  constexpr int WSLAB = XTAPS * NP * NT * 16;    // bytes per weight chunk
  constexpr bool POOL = (MODE == ACT_NORM_POOL);
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_POOL || MODE == ACT_NORM_UP);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  constexpr int NR = POOL ? 4 : 1;
  extern __shared__ __attribute__((aligned(16))) char xsm[];
  const int HP = TH + 2, WP = W + 2;
  const int pixP = HP * WP;
  const int xslab = (pixP + 1) * XPS;   // + one dummy record for out-of-halo items
  char* lw0 = xsm;
  char* lx0 = xsm + 2 * WSLAB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hk = lane >> 5;
  const int tpi = H / TH;
  const int b0 = blockIdx.x / tpi;
  const int h0 = (blockIdx.x % tpi) * TH;
  const int tpx = TH * W;

  // A rows: halo pixel of this lane's output pixel for each m-fragment
  int abase[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int p = wm * MW + mf * 32 + l32;
    const int r = p / W, c = p - r * W;
    abase[mf] = r * WP + c;
  }
  // this lane half's tap of k-step s (tap 9 reads tap 8's pixels; its weights are zero)
  int toff[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int t = min(2 * s + hk, 8);
    toff[s] = (t / 3) * WP + t % 3;
  }

  const int Hs = POOL ? 2 * H : (UPS ? H / 2 : H);
  const int Ws = POOL ? 2 * W : (UPS ? W / 2 : W);
  const float* sb = src + (size_t)b0 * Hs * Ws * Cin;
  const int q = tid & 1;   // this thread's 4-channel half of every 8-channel chunk

  // halo item k: pixel (tid + NTHR*k) >> 1, channels q*4..q*4+3; chunk-invariant source
  // coordinates packed as (gh << 16) | gw, -1 = zero padding / past the halo
  int hw[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    const int pix = (tid + NTHR * k) >> 1;
    const int hh = pix / WP, ww = pix - hh * WP;
    const int gh = h0 + hh - 1, gw = ww - 1;
    hw[k] = (pix < pixP && gh >= 0 && gh < H && gw >= 0 && gw < W) ? ((gh << 16) | gw) : -1;
  }
  float4 raw[KX][NR];
  float2 st[4];
  int cur_ch = 0;
  auto issue_halo = [&](int ch) {   // branch-free: padding items load a safe address
    cur_ch = ch;
    const int c = ch * XCK + q * 4;
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int hv = hw[k] < 0 ? 0 : hw[k];
      const int gh = hv >> 16, gw = hv & 0xffff;
      if (POOL) {
        const float* p = sb + ((size_t)(2 * gh) * Ws + 2 * gw) * Cin + c;
        const size_t rs = (size_t)Ws * Cin;
        raw[k][0] = ld4(p);
        raw[k][NR > 1 ? 1 : 0] = ld4(p + Cin);
        raw[k][NR > 2 ? 2 : 0] = ld4(p + rs);
        raw[k][NR > 3 ? 3 : 0] = ld4(p + rs + Cin);
      } else if (UPS) {
        raw[k][0] = ld4(sb + ((size_t)(gh >> 1) * Ws + (gw >> 1)) * Cin + c);
      } else {
#ifdef EV_X_NOLOAD   // timing experiment only: no halo loads (wrong results)
        raw[k][0] = make_float4((float)gh, (float)gw, 0.f, 1.f);
#else
        raw[k][0] = ld4(sb + ((size_t)gh * Ws + gw) * Cin + c);
#endif
      }
    }
    if (NORM) {
      const float2* s = sstats + (size_t)b0 * Cin + c;
      st[0] = s[0]; st[1] = s[1]; st[2] = s[2]; st[3] = s[3];
    }
  };
  auto store_halo = [&](char* lx) {
    float2 fs[4];
    if (NORM) {
#pragma unroll
      for (int i = 0; i < 4; ++i) fs[i] = norm_fs(st[i]);
    }
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int pix = (tid + NTHR * k) >> 1;
      float4 v = raw[k][0];
      if (POOL)
        v = max4(max4(raw[k][0], raw[k][NR > 1 ? 1 : 0]),
                 max4(raw[k][NR > 2 ? 2 : 0], raw[k][NR > 3 ? 3 : 0]));
      if (NORM)
        v = make_float4(normact_fs(v.x, fs[0]), normact_fs(v.y, fs[1]), normact_fs(v.z, fs[2]),
                        normact_fs(v.w, fs[3]));
      const bool ok = hw[k] >= 0;
      v = make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
      if (act_out) {   // uniform: materialise the (pooled) activation for the wgrad
        const int gh = hw[k] >> 16, gw = hw[k] & 0xffff;
        if (ok && gh >= h0 && gh < h0 + TH)
          st4(act_out + (((size_t)b0 * H + gh) * W + gw) * Cin + cur_ch * XCK + q * 4, v);
      }
      bf16x4 pc[NP];
      split4<NP>(v, pc);
      char* d = lx + (pix < pixP ? pix : pixP) * XPS + q * 8;
#pragma unroll
      for (int i = 0; i < NP; ++i) *reinterpret_cast<bf16x4*>(d + 16 * i) = pc[i];
    }
  };
  auto issue_weights = [&](int ch, char* lw) {
    const char* g = wp + (size_t)ch * WSLAB;
    for (int pc = wave; pc < WSLAB / 1024; pc += NWV)
      __builtin_amdgcn_global_load_lds((const void*)(g + pc * 1024 + lane * 16),
                                       (lds_void_ptr)(lw + pc * 1024), 16, 0, 0);
  };

  f32x16 acc[MF][NF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mf][nf][r] = 0.f;

  const int nchunks = Cin / XCK;
  issue_weights(0, lw0);
  issue_halo(0);
  store_halo(lx0);
  __syncthreads();
  const int ncol = wn * NF * 32 + l32;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int cur = ch & 1, nxt = cur ^ 1;
    const bool more = ch + 1 < nchunks;
    if (more) {
      issue_weights(ch + 1, lw0 + nxt * WSLAB);
      issue_halo(ch + 1);
    }
    const char* lx = lx0 + cur * xslab;
    const char* lw = lw0 + cur * WSLAB;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      bf16x8 a[NP][MF], b[NP][NF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const char* pa = lx + (abase[mf] + toff[s]) * XPS;
#pragma unroll
        for (int i = 0; i < NP; ++i) a[i][mf] = lds_frag(pa + 16 * i);
      }
      const int t = 2 * s + hk;
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        const char* pb = lw + ((t * NP) * NT + ncol + nf * 32) * 16;
#pragma unroll
        for (int i = 0; i < NP; ++i) b[i][nf] = lds_frag(pb + i * NT * 16);
      }
      // terms of total order < NP, smallest first
#ifndef EV_X_NOMFMA   // timing experiment only: no MFMAs (wrong results)
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          if (NP == 3) {
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mf], b[NP - 2][nf], acc[mf][nf], 0, 0, 0);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[NP - 1][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[NP - 1][nf], acc[mf][nf], 0, 0, 0);
          }
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[1][nf], acc[mf][nf], 0, 0, 0);
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
        }
#else
      for (int mf = 0; mf < MF; ++mf)
        for (int nf = 0; nf < NF; ++nf)
          for (int i = 0; i < NP; ++i) acc[mf][nf][i] += (float)a[i][mf][0] * (float)b[i][nf][1];
#endif
    }
    if (more) store_halo(lx0 + nxt * xslab);
    __syncthreads();
  }
  conv_epilogue<MF, NF, FP>(acc, bias, y, spart, B, H, W, NT, b0, h0, tpx, wm * MW, wn * NF * 32, hk,
                            l32, yprev, stprev, ipart);
}

// Workgroup barrier that leaves this wave's N youngest vector-memory operations in flight:
// s_waitcnt vmcnt(N) lgkmcnt(0); s_barrier.  The empty asm "memory" clobbers keep the
// compiler from moving LDS / global accesses across it.
// 1-KiB LDS-DMA pieces per wave and chunk of the pipelined kernel's weight slab
constexpr int pipe_dma_per(int wslab, int nwv) { return (wslab / 1024 + nwv - 1) / nwv; }
// halo items staged at k-step s of the pipelined kernel (item k goes to k-step k*5/KX, or all
// to the last k-step when the prefetch distance is 1)
constexpr int pipe_items_at(int s, int kx, int pd) {
  int n = 0;
  for (int k = 0; k < kx; ++k) n += ((pd == 2 ? (k * 5) / kx : 4) == s) ? 1 : 0;
  return n;
}

// Workgroup barrier with no vector-memory wait (resident-weight kernels: no LDS-DMA in the loop,
// and every register load is waited for by the compiler where it is used): lgkmcnt(0) only
EV_DEVINL void pipe_barrier_lds() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xF | (7 << 4) | (3 << 14));   // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
EV_DEVINL void pipe_barrier() {
  static_assert(N >= 0 && N < 16, "vmcnt range");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(N | (7 << 4));   // vmcnt(N) expcnt(7) lgkmcnt(0) (gfx9 encoding)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Epilogue of conv3x3_pipe_kernel: conv_epilogue (conv_common.h) for one tile of one image,
// with 32-bit buffer offsets instead of 64-bit addresses (the same values, the same
// summation order, so results are bit-identical to the non-persistent kernel's).
//   wpx0  tile pixel of the wave's first fragment, mfs the pixel stride between its fragments
//         (32: one contiguous run; W: FP_POOLOUT's / FP_UPSUM's row pairs), slot the
//         statistics slot of its first 64 pixels: the wave's MF fragments form MF / 2 groups
//         of two (64 pixels) and every group writes one {mean, M2} (spart) or one fused-reduce
//         double2 (ipart) slot, so every configuration has (H*W)/64 slots per image
//   ypool FP_POOLOUT: the (H/2, W/2) max-pooled raw output (2x2 windows are lane-local)
//   Fused input-gradient launches write h = g * lrelu'(xhat), not g (conv_common.h).
//   PH    0: the whole epilogue; with a fused IN-backward reduce of one 32-channel fragment
//         column (pipe_prefetch_ok), PH 1 only loads the tile's y_prev values into pv (issued
//         one iteration early, so their latency hides under that iteration's MFMAs) and PH 2
//         is the epilogue reading them from pv instead of memory (same values, same order)
// cache policy of the epilogue's stream traffic -- the output stores and the fused reduce's
// y_prev loads, each touched once -- non-temporal (CPol NT), so the L2 keeps the halo lines the
// next chunk iterations and tiles re-read instead
#ifndef EV_EPI_POL
#define EV_EPI_POL 2
#endif
constexpr int kEpiPol = EV_EPI_POL;

template <int MF, int NF, int FP>
constexpr bool pipe_prefetch_ok() { return NF == 1 && (FP == P_ID || FP == FP_UPSUM); }
template <int MF, int NF, int FP>
constexpr int pipe_prefetch_n() {
  return pipe_prefetch_ok<MF, NF, FP>() ? (FP == FP_UPSUM ? 8 * (MF / 2) : 16 * MF) : 1;
}
template <int MF, int NF, int FP, int NT, int PH = 0>
EV_DEVINL void pipe_epilogue(f32x16 (&acc)[MF][NF], const float* __restrict__ bias,
                             float* __restrict__ y, float2* __restrict__ spart, int H, int W, int b0,
                             int h0, int wpx0, int mfs, int slot, int co_base, int hk, int l32,
                             const float* __restrict__ yprev, const float2* __restrict__ stprev,
                             double2* __restrict__ ipart, float* __restrict__ ypool, float sc,
                             float (&pv)[pipe_prefetch_n<MF, NF, FP>()]) {
  static_assert(MF % 2 == 0, "fragments in 64-pixel pairs");
  static_assert(PH == 0 || pipe_prefetch_ok<MF, NF, FP>(), "prefetch phases: NF 1, P_ID / UPSUM");
  constexpr int NG = MF / 2;
  // input-gradient launches (a fused IN-backward reduce or the summed upsample adjoint) pass no
  // statistics partials (spart == nullptr)
  constexpr bool FUSED = FP == P_ID || FP == P_POOL || FP == P_UP || FP == FP_UPSUM;
#ifndef EV_EPI_OPAQUE
#define EV_EPI_OPAQUE 1
#endif
  constexpr bool EPI_OPAQUE = EV_EPI_OPAQUE && FP == FP_POOLOUT;
  if constexpr (PH == 1) {   // loads only: the offsets of the PH 0 / 2 code below
    const int nf = 0;
    const int co = co_base + l32;
    if constexpr (FP == FP_UPSUM) {
      const int W2 = W >> 1;
      const auto rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(yprev + ((size_t)b0 * (H >> 1) + (h0 >> 1)) * W2 * NT), 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int m0 = 2 * g;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int prow, pc;
          if (W >= 32) {
            const int r = 2 * k;
            prow = (wpx0 / W + m0) >> 1;
            pc = ((wpx0 % W + 4 * hk) >> 1) + (((r & 3) + 8 * (r >> 2)) >> 1);
          } else {
            const int mf = m0 + (k >> 2), r = 2 * (k & 3);
            prow = (wpx0 + mf * mfs) / W >> 1;
            pc = ((r & 3) + 8 * (r >> 2) + 4 * hk) >> 1;
          }
          pv[g * 8 + k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                        rp, ((prow * W2 + pc) * NT + co) * 4, 0, kEpiPol));
        }
      }
    } else {
      const int lW = 31 - __builtin_clz(W);
      const int plane = H * W;
      const auto rp = __builtin_amdgcn_make_buffer_rsrc((void*)(yprev + (size_t)b0 * plane * NT), 0,
                                                        plane * NT * 4, 0x00020000);
      const int pbase = h0 * W + wpx0 + 4 * hk;
#pragma unroll
      for (int e = 0; e < 16 * MF; ++e) {
        const int mf = e >> 4, r = e & 15;
        const int pl = pbase + mf * 32 + (r & 3) + 8 * (r >> 2);
        pv[e] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rp, (inbwd_pix<FP>(pl, W, lW, 0) * NT + co) * 4, 0, kEpiPol));
      }
    }
    (void)nf;
    return;
  }
  const int T = (H * W) / 64;
  const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)(y + ((size_t)b0 * H + h0) * W * NT), 0,
                                                    0x7fffffff, 0x00020000);
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int co = co_base + nf * 32 + l32;
    const float bb = bias ? bias[co] : 0.f;
    const int vbase = ((wpx0 + 4 * hk) * NT + co) * 4;
    float s[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) s[g] = 0.f;
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        // sc: the exact power-of-two undo of the f16 weight [and gradient] scale, so the fma
        // rounds once, as (acc * sc) + bb did
        const float v = fmaf(acc[mf][nf][r], sc, bb);
        acc[mf][nf][r] = v;
        if constexpr (!FUSED) s[mf >> 1] += v;   // input-gradient convs write no statistics
      }
    // fused input gradients write h (below); pooled inference writes ypool only (one uniform
    // branch, not one per value)
    if (!FUSED && (FP != FP_POOLOUT || y)) {
      // pooled producers: the per-lane store offsets are tile-invariant, and hipcc hoists every
      // one of them out of the tile loop (16 + 8 per fragment column) -- the registers the
      // 64-channel producer then spilled.  An opaque copy of the base keeps them in the epilogue
      // (base + constant, mostly folded into the store's immediate offset)
      int vb = vbase;
      if constexpr (EPI_OPAQUE) asm volatile("" : "+v"(vb));
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          // (a named float: __builtin_bit_cast of the vector-element lvalue itself reads
          // element 0 -- hipcc / ROCm 7.2)
          const float v = acc[mf][nf][r];
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), ry,
                                                vb + (mf * mfs + (r & 3) + 8 * (r >> 2)) * NT * 4, 0, kEpiPol);
        }
    }
    if (FP == FP_UPSUM) {
      // y is (B, H/2, W/2, NT): the 2x2 sums of this conv's output (the upsample adjoint),
      // and the previous block (at H/2) is reduced once per window:
      // sum_window(g) * lrelu'(xhat) == sum_window(g * lrelu'(xhat)), xhat constant on it
      const int W2 = W >> 1;
      const auto rq = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(y + ((size_t)b0 * (H >> 1) + (h0 >> 1)) * W2 * NT), 0, 0x7fffffff, 0x00020000);
      const auto rp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(yprev + ((size_t)b0 * (H >> 1) + (h0 >> 1)) * W2 * NT), 0, 0x7fffffff, 0x00020000);
      const float2 sp = stprev[(size_t)b0 * NT + co];
      const float spc = -sp.x * sp.y;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int m0 = 2 * g;   // the group's fragment pair
        float gs[8], v[8];
        int off[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int prow, pc;
          if (W >= 32) {   // fragment m0 = row 2rp, fragment m0 + 1 = row 2rp + 1, same 32 columns
            const int r = 2 * k;
            gs[k] = (acc[m0][nf][r] + acc[m0][nf][r + 1]) + (acc[m0 + 1][nf][r] + acc[m0 + 1][nf][r + 1]);
            prow = (wpx0 / W + m0) >> 1;
            pc = ((wpx0 % W + 4 * hk) >> 1) + (((r & 3) + 8 * (r >> 2)) >> 1);
          } else {         // W == 16: a fragment is two rows; the window is r, r+1, r+8, r+9
            const int mf = m0 + (k >> 2), r = 2 * (k & 3);
            gs[k] = (acc[mf][nf][r] + acc[mf][nf][r + 1]) + (acc[mf][nf][r + 8] + acc[mf][nf][r + 9]);
            prow = (wpx0 + mf * mfs) / W >> 1;
            pc = ((r & 3) + 8 * (r >> 2) + 4 * hk) >> 1;
          }
          off[k] = ((prow * W2 + pc) * NT + co) * 4;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
          v[k] = PH == 2 ? pv[g * 8 + k]
                         : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rp, off[k], 0, kEpiPol));
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float h = inbwd_acc<P_ID>(gs[k], &v[k], sp, spc, s1, s2);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, h), rq, off[k], 0, kEpiPol);
        }
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (hk == 0) ipart[((size_t)b0 * T + slot + g) * NT + co] = make_double2((double)s1, (double)s2);
      }
    }
    if (FP == FP_POOLOUT) {
      // max(lrelu(IN(y))) over a window == lrelu(IN(max y)) (IN's scale is positive, both maps
      // are monotone), so the consumer reads this tensor in ACT_NORM mode with y's statistics
      const int W2 = W >> 1;
      const auto rq = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(ypool + ((size_t)b0 * (H >> 1) + (h0 >> 1)) * W2 * NT), 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int m0 = 0; m0 < MF; m0 += 2) {
        if (W >= 32) {   // fragment m0 = tile row 2rp, fragment m0 + 1 = row 2rp + 1, same 32 columns
          const int prow = (wpx0 / W + m0) >> 1, pcol = (wpx0 % W + 4 * hk) >> 1;
          int pb = ((prow * W2 + pcol) * NT + co) * 4;
          if constexpr (EPI_OPAQUE) asm volatile("" : "+v"(pb));
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const float m = fmaxf(fmaxf(acc[m0][nf][r], acc[m0][nf][r + 1]),
                                  fmaxf(acc[m0 + 1][nf][r], acc[m0 + 1][nf][r + 1]));
            const int dc = ((r & 3) + 8 * (r >> 2)) >> 1;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, m), rq,
                                                  pb + dc * NT * 4, 0, kEpiPol);
          }
        } else {         // W == 16: a fragment is two rows; the window is r, r+1, r+8, r+9
#pragma unroll
          for (int mf = m0; mf < m0 + 2; ++mf) {
            const int prow = (wpx0 + mf * mfs) / W >> 1;
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
              const float m = fmaxf(fmaxf(acc[mf][nf][r], acc[mf][nf][r + 1]),
                                    fmaxf(acc[mf][nf][r + 8], acc[mf][nf][r + 9]));
              const int pc = ((r & 3) + 8 * (r >> 2) + 4 * hk) >> 1;
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, m), rq,
                                                    ((prow * W2 + pc) * NT + co) * 4, 0, kEpiPol);
            }
          }
        }
      }
    }
    if (FP != FP_NONE && FP != FP_POOLOUT && FP != FP_UPSUM) {
      constexpr int NL = FP == P_POOL ? 4 : 1;
      constexpr int GM = NF == 1 ? 32 : EV_PIPE_EPI_G;   // loads in flight per batch
      constexpr int G = (GM / NL) < 32 ? (GM / NL) : 32;
      static_assert(32 % G == 0, "batches stay inside one 64-pixel group");
      const int lW = 31 - __builtin_clz(W);
      const int plane = FP == P_POOL ? 4 * H * W : (FP == P_UP ? (H * W) / 4 : H * W);
      const auto rp = __builtin_amdgcn_make_buffer_rsrc((void*)(yprev + (size_t)b0 * plane * NT), 0,
                                                        plane * NT * 4, 0x00020000);
      const float2 sp = stprev[(size_t)b0 * NT + co];
      const float spc = -sp.x * sp.y;
      const int pbase = h0 * W + wpx0 + 4 * hk;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e0 = 32 * g; e0 < 32 * g + 32; e0 += G) {
          float v[G][NL];
#pragma unroll
          for (int j = 0; j < G; ++j) {
            const int e = e0 + j, mf = e >> 4, r = e & 15;
            const int pl = pbase + mf * 32 + (r & 3) + 8 * (r >> 2);
#pragma unroll
            for (int k = 0; k < NL; ++k)
              v[j][k] = PH == 2 ? pv[e]
                                : __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                                rp, (inbwd_pix<FP>(pl, W, lW, k) * NT + co) * 4, 0, kEpiPol));
          }
#pragma unroll
          for (int j = 0; j < G; ++j) {
            const int e = e0 + j, mf = e >> 4, r = e & 15;
            const float h = inbwd_acc<FP>(acc[mf][nf][r], v[j], sp, spc, s1, s2);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, h), ry,
                                                  vbase + (mf * mfs + (r & 3) + 8 * (r >> 2)) * NT * 4, 0, kEpiPol);
          }
        }
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (hk == 0) ipart[((size_t)b0 * T + slot + g) * NT + co] = make_double2((double)s1, (double)s2);
      }
    }
    if (!FUSED && spart) {
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        float sg = s[g];
        sg += __shfl_xor(sg, 32, 64);
        const float mean = sg * (1.0f / 64);
        float q = 0.f;
#pragma unroll
        for (int mf = 2 * g; mf < 2 * g + 2; ++mf)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = acc[mf][nf][r] - mean;
            q = fmaf(d, d, q);
          }
        q += __shfl_xor(q, 32, 64);
        if (hk == 0) spart[((size_t)b0 * T + slot + g) * NT + co] = make_float2(mean, q);
      }
    }
  }
}

// WREG (round 6): the one-image 8x8 configuration (4 waves of 64 px x 32 co, one block per CU)
// loads its weight fragments straight into registers (each lane's 16-byte B fragment of every
// k-step, 40 VGPRs per chunk, double-buffered by chunk parity) instead of DMA-ing the 40-KiB
// slab into LDS and reading it back: the four waves need disjoint 32-channel column blocks of
// it, so the LDS round trip carried no reuse, and its writes and reads were half of the
// iteration's LDS traffic (EV_WREG=0: the LDS slab, A/B)
#ifndef EV_WREG
#define EV_WREG 1
#endif
constexpr bool pipe_wreg(int NWV, int WM, int NF, int NI, int WR) {
  return EV_WREG && NWV == 4 && WM == 1 && NF == 1 && NI == 1 && WR == 0;
}

// Persistent, software-pipelined form of conv3x3_split_kernel (same tiles, LDS layouts,
// MFMA sequence and epilogue, so its results are bit-identical).  Each block owns a
// contiguous run of tiles (row bands; consecutive ones are neighbouring bands of one image,
// so their halo rows hit this XCD's L2) and walks the flattened (tile, 8-channel chunk)
// iteration space it = 0 .. ntiles*nch-1 with
//   * the weight slab of it+1 DMA'd into the other LDS buffer (global_load_lds),
//   * the halo of it+PD loaded into a register slot (PD = 2; 1 for max-pool sources, whose
//     four taps per item would not fit twice in VGPRs),
//   * the halo of it+1 transformed (IN + LReLU [+ pool / upsample]), split into bf16 pieces
//     and written to the other LDS buffer item by item BETWEEN the k-steps of it, so the
//     staging VALU work issues while the matrix pipe is busy with it's MFMAs,
//   * one barrier per iteration, and the epilogue of a finished tile run at the start of the
//     next iteration (after the barrier), so its stores drain under the next tile's MFMAs.
// The old kernel paid each of these serially: one exposed global-load latency and one VALU
// staging phase per chunk, plus the prologue / epilogue per tile (tools/conv_micro.py).
//   WR > 0: the layer's WR = Cin / 8 weight slabs are loaded into LDS once, in the prologue,
//   and stay resident (Cin = 32 layers, where they fit beside the halo buffers): no weight
//   DMA per iteration (its issue cost sits in every iteration's instruction stream)
template <int NP, int NWV, int WM, int MF, int NF, int KX, int MODE, int FP, int NI, int WR>
__global__ __launch_bounds__(NWV * 64, (MODE == ACT_FIRST || pipe_wreg(NWV, WM, NF, NI, WR)) ? 1 : 2) void conv3x3_pipe_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, const char* __restrict__ wp,
    const float* __restrict__ bias, float* __restrict__ y, float2* __restrict__ spart,
    float* __restrict__ act_out, int B, int H, int W, int Cin, int TH, int tpb,
    const float* __restrict__ yprev, const float2* __restrict__ stprev, double2* __restrict__ ipart,
    float* __restrict__ ypool, const float* __restrict__ gmax, int gmT, float2* __restrict__ st_out,
    float2* __restrict__ bst_out, double fin_inv_hw, const float* __restrict__ w0,
    const float* __restrict__ b0) {
  constexpr int WN = NWV / WM;
  constexpr int NT = WN * NF * 32;               // == Cout
  constexpr int MW = MF * 32;
  constexpr int NPC = npc(NP);                   // pieces per operand
  constexpr int WSLAB = XTAPS * NPC * NT * 16;
  constexpr int WPER = pipe_dma_per(WSLAB, NWV);  // 1-KiB weight pieces per wave per chunk
  constexpr int WSLABP = WPER * NWV * 1024;       // LDS weight buffer (padded to whole rounds)
  constexpr bool POOL = (MODE == ACT_NORM_POOL);
  // ACT_FIRST: staged like ACT_NORM (statistics, edge-row mask), its pre-norm values computed
  // from x instead of loaded (the block's LDS holds the tile's x rows and the first conv's taps)
  constexpr bool FIRST = (MODE == ACT_FIRST);
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_POOL || MODE == ACT_NORM_UP || FIRST);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  constexpr int NR = POOL ? 4 : 1;
  constexpr bool GS = (NP == NP_F16 && MODE == ACT_RAW);   // per-image gradient scale
  constexpr int PD = POOL ? 1 : 2;               // halo prefetch distance (iterations)
  // vector-memory ops issue_halo makes per iteration: the halo loads and, for NORM sources, the
  // two per-lane loads of the chunk's statistics (the barrier leaves exactly these in flight)
  constexpr int NLD = KX * NR + (NORM ? 2 : 0);
  static_assert(PD == 1 || NLD <= 15, "pipe_barrier: vmcnt range");
  static_assert(WR == 0 || (PD == 2 && NI == 1), "resident weights: single-image, prefetch 2");
  static_assert(!FIRST || (WR > 0 && NI == 1), "ACT_FIRST: the resident-weight single-image form");
  extern __shared__ __attribute__((aligned(16))) char xsm[];
  // a tile is TH rows of one image, or NI whole images (NI > 1: TH == H); NI is a template
  // parameter so the single-image kernels carry none of the per-image bookkeeping
  const int HP = TH + 2, WP = W + 2;
  const int pixI = HP * WP;            // halo pixels per image of the tile
  const int pixP = NI * pixI;
  const int xslab = (pixP + 1) * XPS;
  char* lw0 = xsm;
  char* lx0 = xsm + (WR ? WR * WSLAB : 2 * WSLABP);
  // ACT_FIRST: two x tiles (tile parity) of TH + 4 rows x W + 2 columns (zero columns at -1 and
  // W, zero rows outside the image), then the first conv's tap table
  const int XTS = FIRST ? (TH + 4) * (W + 2) : 0;
  float* xtl = reinterpret_cast<float*>(lx0 + 2 * xslab);
  const float4* wtab = reinterpret_cast<const float4*>(xtl + 2 * XTS);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hk = lane >> 5;
  const int tpi = H / TH;
  const int tpx = TH * W;
  const int nch = Cin / XCK;
  const int t0 = blockIdx.x * tpb;
  const int ntl = min(tpb, ((B + NI - 1) / NI) * tpi - t0);
  const int nit = ntl * nch;

  // the wave's fragments: tile pixel of the first (fpx0) and the stride between them (mfs).
  // FP_POOLOUT on W >= 32 pairs rows (fragment 0 = row 2rp, fragment 1 = row 2rp + 1 of the
  // same 32 columns) so every 2x2 pooling window is lane-local; otherwise one contiguous run
  // (for W == 16 the window is already inside a fragment)
  int fpx0 = wm * MW, mfs = 32;
  if ((FP == FP_POOLOUT || FP == FP_UPSUM) && W >= 32) {
    const int cbs = W >> 5, rp = wm / cbs;
    fpx0 = MF * rp * W + (wm - rp * cbs) * 32;   // rows MF*rp .. MF*rp + MF-1 (pairs)
    mfs = W;
  }
  int abase[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int p = fpx0 + mf * mfs + l32;
    const int im = p / tpx, pr = p - im * tpx;
    const int r = pr / W, c = pr - r * W;
    abase[mf] = im * pixI + r * WP + c;
  }
  int toff[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int t = min(2 * s + hk, 8);
    toff[s] = (t / 3) * WP + t % 3;
  }

  const int Hs = POOL ? 2 * H : (UPS ? H / 2 : H);
  const int Ws = POOL ? 2 * W : (UPS ? W / 2 : W);
  const int q = tid & 1;
  // halo items: image img_w = wave / WPI of the tile is staged by its own WPI waves (so the
  // IN statistics a wave needs are one image's: wave-uniform); half-item hi of the group
  constexpr int WPI = NWV / NI;
  static_assert(NWV % NI == 0, "waves split evenly over the tile's images");
  const int img_w = wave / WPI;
  const int tig = tid - img_w * WPI * 64;
  // tile-invariant item geometry.  Items cover the halo's interior columns only: the two
  // zero-padding columns of every halo row are zeroed in LDS once (zero_pad_columns) and never
  // staged.  hm1 = halo row - 1, boff = the item's byte offset in its source image relative
  // to the tile's first row (0x80000000 = dead item, always out of range), ldo = its LDS
  // record offset (dead items write the dummy record pixP)
  const int NIT = (TH + 2) * W;   // staged items (pixels) per image of the tile
  int hm1[KX], boff[KX], ldo[KX];
  int xoff[FIRST ? KX : 1];        // ACT_FIRST: top-left of the item's 3x3 x window in the x tile
  const int rowb = Ws * Cin * 4;   // bytes per source row
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    const int pixl = (tig + WPI * 64 * k) >> 1;   // interior pixel within this image's halo
    const bool in = pixl < NIT;
    const int hh = pixl / W, c = pixl - hh * W;
    const int r = hh - 1;
    // halo row hh is image row h0 + hh - 1; its window rows h0 + hh - 2 .. h0 + hh are x-tile
    // rows hh .. hh + 2, its columns c - 1 .. c + 1 padded columns c .. c + 2
    if constexpr (FIRST) xoff[k] = in ? hh * (W + 2) + c : 0;
    int o;
    if (POOL) o = 2 * r * rowb + 2 * c * Cin * 4;
    else if (UPS) o = (r >> 1) * rowb + (c >> 1) * Cin * 4;
    else o = r * rowb + c * Cin * 4;
    hm1[k] = in ? r : -(1 << 28);
    boff[k] = in ? o + img_w * (Hs * Ws * Cin * 4) + q * 16 : (int)0x80000000;
    ldo[k] = (in ? img_w * pixI + hh * WP + c + 1 : pixP) * XPS + q * 8;
  }
  const int img_bytes = Hs * Ws * Cin * 4;
  // item k of this wave holds at least one halo pixel (wave index made provably uniform so
  // the test is a scalar branch)
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const int tig_u = __builtin_amdgcn_readfirstlane(tig - (tid & 63));   // the wave's first lane
  const int img_u = __builtin_amdgcn_readfirstlane(img_w);
  auto item_live = [&](int k) EV_LAMBDA_INLINE { return (tig_u + WPI * 64 * k) < 2 * NIT; };
  // Halo rows above / below the image: their loads fall outside the buffer range and read 0,
  // which is the right value for RAW sources of one-image tiles; the NORM transform of 0 is
  // not 0, and with two images per tile a row outside one image is inside the other, so those
  // stage through a row mask -- only on tiles at the top / bottom of the image (scalar flag)
  constexpr bool MASK = NORM || NI > 1;
  float4 raw[PD][KX][NR];
  float2 st[PD][4];
  int edge[PD];                    // MASK: the slot's tile touches the image top / bottom
  int sb0[PD], sh0[PD], sch[PD];   // tile image / first row / chunk of the slot's data
  float gsc[PD];                   // GS: the slot image's gradient scale
  int sxb[PD];                     // ACT_FIRST: x-tile buffer (tile parity) of the slot's tile
  constexpr int XTN = 4;           // ACT_FIRST: x-tile elements per thread (TH + 4) * (W + 2) / threads
  float xtr[XTN];
  int xt_pend = -1;                // ACT_FIRST: x-tile buffer to write at the end of the iteration
  auto load_xtile = [&](int b, int h0) EV_LAMBDA_INLINE {
    const float* xb = src + (size_t)b * H * W;
#pragma unroll
    for (int j = 0; j < XTN; ++j) {
      const int i = tid + NWV * 64 * j;
      const int r = i / (W + 2), cc = i - r * (W + 2);
      const int gh = h0 - 2 + r, gw = cc - 1;
      xtr[j] = (i < XTS && gh >= 0 && gh < H && gw >= 0 && gw < W) ? xb[gh * W + gw] : 0.f;
    }
  };
  auto store_xtile = [&](int buf) EV_LAMBDA_INLINE {
#pragma unroll
    for (int j = 0; j < XTN; ++j) {
      const int i = tid + NWV * 64 * j;
      if (i < XTS) xtl[buf * XTS + i] = xtr[j];
    }
  };
  int gs_b = -1;                   // GS: image whose shift gs_k holds
  int gs_k = 0;
  auto gshift = [&](int b) EV_LAMBDA_INLINE {
    if (b != gs_b) { gs_b = b; gs_k = f16_gshift(gmax, gmT, b); }
    return gs_k;
  };

  // nch, H and TH are powers of two (plan_split), so the iteration -> (image, row, chunk) map
  // is shifts and masks: no runtime integer division (a ~30-instruction SALU chain each) in
  // the per-iteration instruction stream
  const int lgnch = 31 - __builtin_clz(nch), lgH = 31 - __builtin_clz(H);
  auto coords = [&](int it, int& b0, int& h0, int& ch) EV_LAMBDA_INLINE {
    const int t = t0 + (it >> lgnch);
    ch = it & (nch - 1);
    if constexpr (NI == 1) {   // tile t = rows t*TH .. of the stacked images
      const int r = t * TH;
      b0 = r >> lgH;
      h0 = r & (H - 1);
    } else {                   // TH == H: tile t = images t*NI ..
      b0 = t * NI;
      h0 = 0;
    }
  };
  // halo loads of iteration it into register slot sl: buffer loads with 32-bit offsets into
  // the tile's source image; rows above / below the image fall outside the descriptor's range
  // and read 0 without touching memory (the NORM transform is masked by okm at staging)
  auto issue_halo = [&](int it, auto slot_c) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(slot_c)::value;
    int b0, h0, ch;
    coords(it, b0, h0, ch);
    sb0[sl] = b0; sh0[sl] = h0; sch[sl] = ch;
    // GS: the scale of the image this wave stages (NI > 1: one image per wave group)
    if constexpr (GS) gsc[sl] = ldexpf(1.f, gshift(NI == 1 ? b0 : min(b0 + img_u, B - 1)));
    if constexpr (MASK) edge[sl] = NI > 1 || h0 == 0 || h0 + TH >= H;
    if constexpr (FIRST) {
      sxb[sl] = (it >> lgnch) & 1;
      // a new tile's x rows: loaded now, written to its parity buffer at the end of this
      // iteration, read from the next iteration's staging on (the prologue writes tile 0's)
      if (ch == 0 && it > 0) {
        load_xtile(b0, h0);
        xt_pend = sxb[sl];
      }
    } else {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)b0 * Hs * Ws * Cin), 0,
                                                      NI == 1 ? img_bytes : img_bytes * min(NI, B - b0),
                                                      0x00020000);
#ifdef EV_X_CONTIG
    const int toff = h0 * rowb + ch * (pixP * 32);
#else
    const int toff = (POOL ? 2 * h0 : (UPS ? (h0 >> 1) : h0)) * rowb + ch * XCK * 4;
#endif
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int vo = boff[k] + toff;
      if (POOL) {
        raw[sl][k][0] = bload4(rs, vo);
        raw[sl][k][NR > 1 ? 1 : 0] = bload4(rs, vo + Cin * 4);
        raw[sl][k][NR > 2 ? 2 : 0] = bload4(rs, vo + rowb);
        raw[sl][k][NR > 3 ? 3 : 0] = bload4(rs, vo + rowb + Cin * 4);
      } else {
        raw[sl][k][0] = bload4(rs, vo);
      }
    }
    }   // !FIRST
    if (NORM) {
      // each lane loads the {mean, rstd} of its own 4-channel half (two 16-byte vector loads;
      // a wave-uniform scalar load would need 3 VALU per value to hand each lane its half)
      const int bs = NI == 1 ? b0 : min(b0 + img_u, B - 1);   // this wave's image
      const float4* sp = reinterpret_cast<const float4*>(sstats + (size_t)bs * Cin + ch * XCK + q * 4);
      const float4 u0 = sp[0], u1 = sp[1];
      st[sl][0] = make_float2(u0.x, u0.y); st[sl][1] = make_float2(u0.z, u0.w);
      st[sl][2] = make_float2(u1.x, u1.y); st[sl][3] = make_float2(u1.z, u1.w);
    }
  };
  // transform + split item k of register slot sl into the LDS halo buffer lx
  // Branch-free so that a k-step's staging and MFMAs form one scheduling region the
  // compiler can interleave (the edge-row mask and the activation hand-off run afterwards,
  // in stage_post, behind uniform branches).
  auto stage_value = [&](auto slot_c, int k, const float2 (&fs)[4]) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(slot_c)::value;
    float4 v = raw[sl][k][0];
    if (POOL)
      v = max4(max4(raw[sl][k][0], raw[sl][k][NR > 1 ? 1 : 0]),
               max4(raw[sl][k][NR > 2 ? 2 : 0], raw[sl][k][NR > 3 ? 3 : 0]));
    if (NORM)
      v = make_float4(normact_fs(v.x, fs[0]), normact_fs(v.y, fs[1]), normact_fs(v.z, fs[2]),
                      normact_fs(v.w, fs[3]));
    return v;
  };
  float4 wq[FIRST ? 10 : 1];   // ACT_FIRST: taps 0..8 and the bias of the staged chunk half
  auto stage_item = [&](auto slot_c, int k, const float2 (&fs)[4], char* lx) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(slot_c)::value;
    float4 v;
    if constexpr (FIRST) {
      // y0 at the item's pixel for its 4 channels: ebsdvae_conv_first_fwd's own fma chain
      // (first_conv_px2 per channel pair), then the same normalisation as ACT_NORM
      const float* xw = xtl + sxb[sl] * XTS + xoff[k];
      float nb[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) nb[t] = xw[(t / 3) * (W + 2) + t % 3];
#ifdef EV_FIRST_PK   // A/B: the channel pairs on v_pk_fma_f32 (first_conv_px2)
      pkf2 wa[9], wb[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        wa[t] = pk2(wq[t].x, wq[t].y);
        wb[t] = pk2(wq[t].z, wq[t].w);
      }
      const pkf2 ya = first_conv_px2(nb, wa, pk2(wq[9].x, wq[9].y));
      const pkf2 yb = first_conv_px2(nb, wb, pk2(wq[9].z, wq[9].w));
      v = make_float4(normact_fs(ya.x, fs[0]), normact_fs(ya.y, fs[1]), normact_fs(yb.x, fs[2]),
                      normact_fs(yb.y, fs[3]));
#else
      // scalar v_fma_f32 chains (a packed fma beside MFMAs costs more issue than two scalar
      // ones, MI355X_MICROARCH.md); each lane of first_conv_px2 is exactly this chain
      float wc[4][9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        wc[0][t] = wq[t].x; wc[1][t] = wq[t].y; wc[2][t] = wq[t].z; wc[3][t] = wq[t].w;
      }
      v = make_float4(normact_fs(first_conv_px(nb, wc[0], wq[9].x), fs[0]),
                      normact_fs(first_conv_px(nb, wc[1], wq[9].y), fs[1]),
                      normact_fs(first_conv_px(nb, wc[2], wq[9].z), fs[2]),
                      normact_fs(first_conv_px(nb, wc[3], wq[9].w), fs[3]));
#endif
    } else {
      v = stage_value(slot_c, k, fs);
    }
    bf16x4 pc[NPC];
    if constexpr (GS)   // the per-image gradient scale folded into the split
      split4_f16_scaled(v, gsc[sl], pc);
    else
      split4<NP>(v, pc);
    char* d = lx + ldo[k];
#pragma unroll
    for (int i = 0; i < NPC; ++i) *reinterpret_cast<bf16x4*>(d + 16 * i) = pc[i];
  };
  // after a halo buffer is staged (same wave, so ordered after its own writes): zero the
  // records of halo rows outside the image (top / bottom tiles, every two-image tile), and
  // materialise the (pooled) activation for the weight gradient when asked to (act_out)
  auto stage_post = [&](auto slot_c, const float2 (&fs)[4], char* lx) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(slot_c)::value;
    if constexpr (MASK) {
      if (edge[sl]) {
#pragma unroll
        for (int k = 0; k < KX; ++k)
          if ((unsigned)(sh0[sl] + hm1[k]) >= (unsigned)H) {
            char* d = lx + ldo[k];
#pragma unroll
            for (int i = 0; i < NPC; ++i) *reinterpret_cast<bf16x4*>(d + 16 * i) = bf16x4{};
          }
      }
    }
    if (act_out) {
#pragma unroll
      for (int k = 0; k < KX; ++k) {
        const int pixl = (tig + WPI * 64 * k) >> 1;
        const int hh = pixl / W, gw = pixl - hh * W;
        if (pixl < NIT && hh >= 1 && hh <= TH && (NI == 1 || sb0[sl] + img_w < B))
          st4(act_out + (((size_t)(sb0[sl] + img_w) * H + sh0[sl] + hh - 1) * W + gw) * Cin +
                  sch[sl] * XCK + q * 4, stage_value(slot_c, k, fs));
      }
    }
  };
  auto stage_fs = [&](auto slot_c, float2 (&fs)[4]) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(slot_c)::value;
#pragma unroll
    for (int i = 0; i < 4; ++i) fs[i] = NORM ? norm_fs(st[sl][i]) : make_float2(1.f, 0.f);
    if constexpr (FIRST) {
      const float4* wt = wtab + (sch[sl] * 2 + q) * 10;
#pragma unroll
      for (int t = 0; t < 10; ++t) wq[t] = wt[t];
    }
  };
  // weight slab DMA: every wave issues exactly WPER 1-KiB pieces per chunk (the padding
  // pieces of the last chunk fall outside the descriptor's range), so every iteration issues
  // the same, compile-time number of vector-memory ops and the compiler's waits stay exact
  const auto rwp = __builtin_amdgcn_make_buffer_rsrc((void*)wp, 0, nch * WSLAB, 0x00020000);
  // NP_F16: the layer's weight shift k (weights packed as w * 2^k), in the pack's trailer
  const int wshift = NP == NP_F16 ? *reinterpret_cast<const int*>(wp + (size_t)nch * WSLAB) : 0;
  constexpr bool WREG = pipe_wreg(NWV, WM, NF, NI, WR);
  bf16x8 wreg[WREG ? 2 : 1][WREG ? 5 : 1][NPC];
  auto issue_wreg = [&](int it, auto slot_c) EV_LAMBDA_INLINE {
    constexpr int sl = decltype(slot_c)::value;
    const int ch = it & (nch - 1);
    const int nc = wn * NF * 32 + l32;   // this lane's output channel (B fragment column)
#pragma unroll
    for (int s5 = 0; s5 < 5; ++s5) {
      const int t = 2 * s5 + hk;
#pragma unroll
      for (int i = 0; i < NPC; ++i)
        wreg[sl][s5][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                          rwp, ch * WSLAB + ((t * NPC + i) * NT + nc) * 16, 0, 0));
    }
  };
  auto issue_weights = [&](int it, char* lw) EV_LAMBDA_INLINE {
    if constexpr (WR || WREG) return;   // resident since the prologue / in registers
    const int ch = it & (nch - 1);
#pragma unroll
    for (int j = 0; j < WPER; ++j) {
      const int pc = wave_u + j * NWV;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwp, (lds_void_ptr)(lw + pc * 1024), 16,
                                               ch * WSLAB + pc * 1024 + lane * 16, 0, 0, 0);
    }
  };

  f32x16 acc[MF][NF];
  auto zero_acc = [&]() EV_LAMBDA_INLINE {
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mf][nf][r] = 0.f;
  };
  const int ncol = wn * NF * 32 + l32;
  // fused IN-backward reduce of one fragment column: the tile's y_prev values are loaded at the
  // start of its last iteration (pipe_epilogue PH 1) and consumed by its epilogue (PH 2)
#ifdef EV_PIPE_NOPREF   // A/B: load them inside the epilogue
  constexpr bool PREF = false;
#else
  constexpr bool PREF = pipe_prefetch_ok<MF, NF, FP>() && NI == 1;
#endif
  float pv[pipe_prefetch_n<MF, NF, FP>()];
  auto epi_prefetch = [&](int it) EV_LAMBDA_INLINE {
    int b0, h0, ch;
    coords(it, b0, h0, ch);
    pipe_epilogue<MF, NF, FP, NT, PREF ? 1 : 0>(acc, bias, y, spart, H, W, b0, h0, fpx0, mfs, 0,
                                                wn * NF * 32, hk, l32, yprev, stprev, ipart, ypool, 1.f, pv);
  };
  auto epilogue = [&](int it_done, f32x16 (&ea)[MF][NF]) EV_LAMBDA_INLINE {
    int b0, h0, ch;
    coords(it_done, b0, h0, ch);
    const int im = NI == 1 ? 0 : (wm * MW) / tpx;   // the wave's pixels lie in one image
    const int wpx0 = fpx0 - im * tpx;
    float sc = 1.f;
    if constexpr (NP == NP_F16) {   // undo the weight [and gradient] scale (powers of two)
      sc = ldexpf(1.f, -wshift);
      if constexpr (GS) sc = ldexpf(sc, -gshift(min(b0 + im, B - 1)));
    }
#ifdef EV_PIPE_NOEPI   // timing experiment only: no epilogue (no output, wrong results)
    if (sc == 12345.f)
#else
    if (NI == 1 || b0 + im < B)
#endif
      pipe_epilogue<MF, NF, FP, NT, PREF ? 2 : 0>(ea, bias, y, spart, H, W, b0 + im, h0, wpx0, mfs,
                                                  (h0 * W + wm * MW - im * tpx) / 64, wn * NF * 32, hk,
                                                  l32, yprev, stprev, ipart, ypool, sc, pv);
  };

#ifdef EV_PIPE_TRACE
  unsigned long long tr_issue = 0, tr_k = 0, tr_bar = 0, tr_epi = 0;
  const unsigned long long tr_start = __builtin_amdgcn_s_memtime();
  const unsigned long long tr_rstart = __builtin_amdgcn_s_memrealtime();
#endif
  // one pipelined iteration; P = it & 1 selects the LDS buffers and register slots statically
  auto body = [&](int it, auto P_c) EV_LAMBDA_INLINE {
    constexpr int P = decltype(P_c)::value;
    constexpr int SL_LD = PD == 2 ? P : 0;        // slot receiving it+PD
    constexpr int SL_ST = PD == 2 ? 1 - P : 0;    // slot holding it+1
    EV_T(tb0);
    // unconditional issue (indices clamped at the end: the surplus loads land in buffers
    // nobody reads), so every iteration has the same vector-memory op count
    const int it1 = min(it + 1, nit - 1), itp = min(it + PD, nit - 1);
    // the tile's last iteration (nch is even, so it is always a P = 1 one): its epilogue's
    // y_prev loads go first, older than this iteration's halo loads, so the barrier's
    // vmcnt(KX) retires them
    if constexpr (PREF && P == 1)
      if ((it & (nch - 1)) == nch - 1) epi_prefetch(it);
#ifndef EV_PIPE_LATE_ISSUE
    issue_weights(it1, lw0 + (1 - P) * WSLABP);
    if constexpr (WREG) issue_wreg(it1, std::integral_constant<int, WREG ? 1 - P : 0>());
    issue_halo(itp, std::integral_constant<int, SL_LD>());
#endif
    EV_TACC(tr_issue, tb0);
    EV_T(tb1);
    float2 fs[4];
    stage_fs(std::integral_constant<int, SL_ST>(), fs);
    const char* lx = lx0 + P * xslab;
    const char* lw = WR ? lw0 + (it & (nch - 1)) * WSLAB : lw0 + P * WSLABP;
    char* lxn = lx0 + (1 - P) * xslab;
    // NF == 1: fragments of k-step s live in register set s & 1, the LDS reads of k-step s+1
    // are issued before the MFMAs of k-step s, so only k-step 0 waits on an LDS latency.
    // NF > 1 has twice the MFMAs per k-step to cover the reads and no VGPRs to spare for a
    // second set (it would spill): one set, read at the start of each k-step
    constexpr bool FPF = NF == 1 && MF <= 2;   // MF = 4 has no VGPRs for a second set
    bf16x8 fa[FPF ? 2 : 1][NPC][MF], fb[FPF ? 2 : 1][NPC][NF];
    auto load_frags = [&](int s, bf16x8 (&a)[NPC][MF], bf16x8 (&b)[NPC][NF]) EV_LAMBDA_INLINE {
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const char* pa = lx + (abase[mf] + toff[s]) * XPS;
#pragma unroll
        for (int i = 0; i < NPC; ++i) a[i][mf] = lds_frag(pa + 16 * i);
      }
      if constexpr (WREG) {
#pragma unroll
        for (int i = 0; i < NPC; ++i) b[i][0] = wreg[WREG ? P : 0][WREG ? s : 0][i];
      } else {
        const int t = 2 * s + hk;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const char* pb = lw + ((t * NPC) * NT + ncol + nf * 32) * 16;
#pragma unroll
          for (int i = 0; i < NPC; ++i) b[i][nf] = lds_frag(pb + i * NT * 16);
        }
      }
    };
    if constexpr (FPF) load_frags(0, fa[0], fb[0]);
    auto kstep = [&](auto s_c) EV_LAMBDA_INLINE {
      constexpr int s = decltype(s_c)::value;
      constexpr int fs_ = FPF ? (s & 1) : 0;
      if constexpr (FPF) {
        if constexpr (s + 1 < 5) load_frags(s + 1, fa[(s + 1) & 1], fb[(s + 1) & 1]);
      } else {
        load_frags(s, fa[0], fb[0]);
      }
      bf16x8 (&a)[NPC][MF] = fa[fs_];
      bf16x8 (&b)[NPC][NF] = fb[fs_];
#if defined(EV_PIPE_NOMFMA2)   // timing experiment only: no MFMA at all, the fragments kept live
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf)
          acc[mf][nf][0] += (float)a[0][mf][0] * (float)b[0][nf][0] + (float)a[1][mf][1] * (float)b[1][nf][1];
#elif !defined(EV_PIPE_NOMFMA)   // timing experiment only: one MFMA per fragment pair (wrong results)
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          if constexpr (NP == 3) {
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mf], b[NP - 2][nf], acc[mf][nf], 0, 0, 0);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[NP - 1][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[NP - 1][nf], acc[mf][nf], 0, 0, 0);
          }
          acc[mf][nf] = mfma_piece<NP>(a[1][mf], b[0][nf], acc[mf][nf]);
          acc[mf][nf] = mfma_piece<NP>(a[0][mf], b[1][nf], acc[mf][nf]);
          acc[mf][nf] = mfma_piece<NP>(a[0][mf], b[0][nf], acc[mf][nf]);
        }
#else
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = mfma_piece<NP>(a[0][mf] + a[1][mf], b[0][nf] + b[1][nf], acc[mf][nf]);
#endif
#ifdef EV_PIPE_LATE_ISSUE
      if (s == 0) {   // behind the first k-step's MFMAs, so the matrix pipe covers the issue
        issue_weights(it1, lw0 + (1 - P) * WSLABP);
        issue_halo(itp, std::integral_constant<int, SL_LD>());
      }
#endif
      // staging of it+1, spread over the k-steps (PD = 1: its loads were issued this
      // iteration, so stage after the last k-step's MFMAs are queued)
#ifndef EV_PIPE_NOSTAGE   // timing experiment only: no staging VALU (wrong results)
      // every item is staged (dead ones load nothing and write the dummy record), so the
      // region has no branch
#pragma unroll
      for (int k = 0; k < KX; ++k)
        if ((PD == 2 ? (k * 5) / KX : 4) == s)
          stage_item(std::integral_constant<int, SL_ST>(), k, fs, lxn);
#endif
#ifdef EV_PIPE_GROUPS   // experiment: measured slower for the input-gradient convs
      // interleave: the next k-step's fragment reads, then each MFMA followed by its share of
      // the staging VALU, so the vector work issues in the matrix pipe's shadow
      {
        constexpr int NMF = MF * NF * (NP == 3 ? 6 : 3);
        constexpr int NIS = pipe_items_at(s, KX, PD);
        constexpr int VPI = (NORM ? 12 : 0) + (POOL ? 12 : 0) + (GS ? 4 : 0) + (NPC == 2 ? 6 : 12);
        constexpr int VPM = (NIS * VPI + NMF - 1) / NMF;
        if constexpr (FPF && s + 1 < 5)
          __builtin_amdgcn_sched_group_barrier(0x100, NPC * (MF + NF), 0);   // DS reads
#pragma unroll
        for (int i = 0; i < NMF; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                   // MFMA
          if (VPM) __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);       // VALU
        }
      }
#endif
#ifndef EV_PIPE_NO_SCHED_FENCE
      __builtin_amdgcn_sched_barrier(0);   // one scheduling region per k-step (VGPR budget)
#endif
    };
    kstep(std::integral_constant<int, 0>());
    kstep(std::integral_constant<int, 1>());
    kstep(std::integral_constant<int, 2>());
    kstep(std::integral_constant<int, 3>());
    kstep(std::integral_constant<int, 4>());
    stage_post(std::integral_constant<int, SL_ST>(), fs, lxn);
    if constexpr (FIRST) {
      if (xt_pend >= 0) {   // the next tile's x rows, before the barrier that publishes them
        store_xtile(xt_pend);
        xt_pend = -1;
      }
    }
    EV_TACC(tr_k, tb1);
    EV_T(tb2);
#ifdef EV_PIPE_NOBAR   // timing experiment only: no barrier (LDS races, wrong results)
    if (false) {
#else
    if (PD == 2) {
#endif
      // the halo loads of it+2 (this wave's youngest vector-memory ops) stay in flight across
      // the barrier: everything older -- the weight DMA of it+1, epilogue traffic -- is retired
      // (resident weights: no DMA to wait for)
      if constexpr (WR > 0)
        pipe_barrier_lds();
      else
        pipe_barrier<(PD == 2 ? NLD : 0)>();
    } else {
#ifndef EV_PIPE_NOBAR
      __syncthreads();
#endif
    }
    EV_TACC(tr_bar, tb2);
  };

#ifdef EV_PIPE_PRIO
  // the younger half of the workgroup loses VALU arbitration to the older half on every
  // segment (MI355X_MICROARCH.md, two waves per SIMD): raise it once
  if (wave_u >= NWV / 2) __builtin_amdgcn_s_setprio(1);   // scalar branch: this wave only
#endif
  // the zero-padding columns of both halo buffers (never staged; every chunk and tile of the
  // block has them at the same records): 16-B granules of the NPC piece slots
  {
    const int nrec = 2 * NI * (TH + 2) * 2;   // buffer x image x halo row x {left, right}
    for (int i = tid; i < nrec * NPC; i += NWV * 64) {
      const int rec = i / NPC, pc = i - rec * NPC;
      const int side = rec & 1, row = (rec >> 1) % (TH + 2), rest = (rec >> 1) / (TH + 2);
      const int img = rest % NI, buf = rest / NI;
      char* d = lx0 + buf * xslab + (img * pixI + row * WP + side * (W + 1)) * XPS + 16 * pc;
      *reinterpret_cast<float4*>(d) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if constexpr (FIRST) {
    // the first conv's taps and bias per (chunk, 4-channel half): [grp][tap 0..8, bias][4]
    float* wtf = reinterpret_cast<float*>(xtl + 2 * XTS);
    for (int i = tid; i < FIRST_WTAB; i += NWV * 64) {
      const int grp = i / 40, rem = i - grp * 40, t = rem >> 2, c = grp * 4 + (rem & 3);
      wtf[i] = t < 9 ? w0[c * 9 + t] : (b0 ? b0[c] : 0.f);
    }
    int xb0, xh0, xch;
    coords(0, xb0, xh0, xch);
    load_xtile(xb0, xh0);
    store_xtile(0);
    __syncthreads();
  }
  // prologue: weights + halo of it 0 (and the halo of it 1 for PD = 2)
  zero_acc();
  if constexpr (WR) {
    // every chunk's slab, 1-KiB pieces over the waves (WR * WSLAB is whole pieces)
    for (int pc = wave_u; pc < WR * WSLAB / 1024; pc += NWV)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwp, (lds_void_ptr)(lw0 + pc * 1024), 16,
                                               pc * 1024 + lane * 16, 0, 0, 0);
  } else if constexpr (WREG) {
    issue_wreg(0, std::integral_constant<int, 0>());
  } else {
    issue_weights(0, lw0);
  }
  issue_halo(0, std::integral_constant<int, 0>());
  {
    float2 fs[4];
    stage_fs(std::integral_constant<int, 0>(), fs);
    if (PD == 2) issue_halo(min(1, nit - 1), std::integral_constant<int, PD == 2 ? 1 : 0>());
#pragma unroll
    for (int k = 0; k < KX; ++k)
      if (item_live(k)) stage_item(std::integral_constant<int, 0>(), k, fs, lx0);
    stage_post(std::integral_constant<int, 0>(), fs, lx0);
  }
  if constexpr (WR) {
    // the resident slabs are older than both halo loads: all but the youngest (it 1's) landed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD) : "memory");
  }
  __syncthreads();
  // nch = Cin / 8 is even for every supported layer (plan_split), so it & 1 == ch & 1
  for (int tl = 0; tl < ntl; ++tl) {
    for (int ch = 0; ch < nch; ch += 2) {
      body(tl * nch + ch, std::integral_constant<int, 0>());
      body(tl * nch + ch + 1, std::integral_constant<int, 1>());
    }
    // after the tile's last barrier: the stores drain under the next tile's MFMAs
    EV_T(te0);
    epilogue(tl * nch, acc);
    zero_acc();
    EV_TACC(tr_epi, te0);
  }
  // InstanceNorm finalize of the images this block owns (the host passes st_out / bst_out
  // only when every block's tile run covers whole images, pipe_owns_images): the forward
  // {mean, rstd} from this conv's statistics partials, or the previous block's backward
  // {m1, m2} from the fused reduce's partials, as the standalone finalize kernels compute them
  if (st_out || bst_out) {
    // the surplus weight DMA of the last iterations still targets LDS, which the finalize
    // reuses; the epilogue stores of every wave must be visible to the whole block
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __threadfence_block();
    __syncthreads();
    const int tpi = NI == 1 ? H / TH : 1;
    const int g0 = t0 / tpi, g1 = (t0 + ntl - 1) / tpi;
    for (int gi = g0; gi <= g1; ++gi)
      for (int im = 0; im < NI; ++im) {
        const int b = gi * NI + im;
        if (b >= B) break;
        if (st_out)
          in_stats_finalize_image(spart, st_out, NT, (H * W) / 64, 64.f, b, tid,
                                  reinterpret_cast<float*>(xsm));
        if (bst_out)
          in_bwd_finalize_image(ipart, bst_out, NT, (H * W) / 64, fin_inv_hw, b, tid,
                                reinterpret_cast<double*>(xsm));
      }
  }
#ifdef EV_PIPE_TRACE
  if (lane == 0 && blockIdx.x < 4096) {
    unsigned long long* o = ev_pipe_trace + ((size_t)blockIdx.x * 8 + (wave & 7)) * 6;
    o[0] = __builtin_amdgcn_s_memtime() - tr_start;
    o[1] = tr_issue; o[2] = tr_k; o[3] = tr_bar; o[4] = tr_epi;
    o[5] = __builtin_amdgcn_s_memrealtime() - tr_rstart;   // 100 MHz
  }
#endif
}

// NP_F16 packs, step 1: partial maxima of |w| per layer, kF16MaxParts blocks per layer, into
// the pack's trailer after its 16-byte head (grid (kF16MaxParts, layers); runs before
// pack_split_kernel on the same stream)
__global__ __launch_bounds__(256) void pack_wmax_kernel(const PackBatch pb) {
  const ebsdvae_pack_desc& q = pb.d[blockIdx.y];
  const int n = q.cin * q.cout * 9;
  float m = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += kF16MaxParts * 256) m = fmaxf(m, fabsf(q.src[i]));
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ci_ = q.for_dgrad ? q.cout : q.cin, co_ = q.for_dgrad ? q.cin : q.cout;
    const size_t body = (size_t)(ci_ / XCK) * XTAPS * npc(NP_F16) * co_ * XCK * 2;
    float* parts = reinterpret_cast<float*>(reinterpret_cast<char*>(q.dst) + body + 16);
    parts[blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
  }
}

// split weight pack: [chunk][tap 0..9][piece][co'][8 ci'] bf16 of the conv-equivalent
// weight (tap 9 = 0); (ci', co') = (cin, cout) of the layer, swapped for the input gradient.
__global__ void pack_split_kernel(const PackBatch pb, int np) {
  const ebsdvae_pack_desc& q = pb.d[blockIdx.y];
  const int ci_ = q.for_dgrad ? q.cout : q.cin;
  const int co_ = q.for_dgrad ? q.cin : q.cout;
  const int nch = ci_ / XCK;
  const int n = nch * XTAPS * co_ * XCK;
  __bf16* d = reinterpret_cast<__bf16*>(q.dst);
  // NP_F16: the layer's weight shift k = f16_shift_of(max |w|) from the partial maxima in the
  // trailer (every block reduces them; block 0 writes k into the 16-byte head, which no block
  // reads, so the order of the blocks does not matter)
  int k16 = 0;
  if (np == NP_F16) {
    const float* parts = reinterpret_cast<const float*>(d + (size_t)n * npc(np)) + 4;
    float m = 0.f;
    for (int i = 0; i < kF16MaxParts; ++i) m = fmaxf(m, parts[i]);
    k16 = m > 0.f ? f16_shift_of(m) : 0;
    if (blockIdx.x == 0 && threadIdx.x == 0)
      *reinterpret_cast<int4*>(d + (size_t)n * npc(np)) = make_int4(k16, 0, 0, 0);
  }
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c8 = e % XCK;
    int r = e / XCK;
    const int o = r % co_;
    r /= co_;
    const int t = r % XTAPS, chunk = r / XTAPS;
    float w = 0.f;
    if (t < 9) {
      const int i = chunk * XCK + c8;
      const int co = q.for_dgrad ? i : o;
      const int ci = q.for_dgrad ? o : i;
      size_t idx;
      if (q.kind == 0) idx = ((size_t)co * q.cin + ci) * 9 + (q.for_dgrad ? 8 - t : t);
      else idx = ((size_t)ci * q.cout + co) * 9 + (q.for_dgrad ? t : 8 - t);
      w = q.src[idx];
    }
    const size_t base = ((size_t)(chunk * XTAPS + t) * npc(np)) * co_ * XCK + (size_t)o * XCK + c8;
    if (np == NP_F16) {   // two fp16 pieces of the scaled weight (conv3x3_pipe_kernel undoes it)
      const float ws = ldexpf(w, k16);
      const _Float16 h0 = (_Float16)ws;
      const _Float16 h1 = (_Float16)(ws - (float)h0);
      d[base] = __builtin_bit_cast(__bf16, h0);
      d[base + (size_t)co_ * XCK] = __builtin_bit_cast(__bf16, h1);
      continue;
    }
    float rr = w;
    for (int i = 0; i < np; ++i) {
      const __bf16 p = (__bf16)rr;
      rr -= (float)p;
      d[base + (size_t)i * co_ * XCK] = p;
    }
  }
}

// EBSDVAE_CONV_PIPE=0 selects the non-persistent conv3x3_split_kernel (A/B timing)
static bool use_pipe() {
  static const int v = [] {
    const char* e = getenv("EBSDVAE_CONV_PIPE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v != 0;
}

// EBSDVAE_CONV_MULTI_IMAGE=0: 8x8 maps go to the fp32 small-map kernels (A/B timing)
// EBSDVAE_CONV_SMALL1=0: the 8x8 split-fp16 convs keep two-image tiles (A/B)
static bool use_small_one_image() {
  static const bool v = [] {
    const char* e = getenv("EBSDVAE_CONV_SMALL1");
    return !(e && e[0] == '0');
  }();
  return v;
}

static bool use_multi_image() {
  static const int v = [] {
    const char* e = getenv("EBSDVAE_CONV_MULTI_IMAGE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v != 0;
}

// EBSDVAE_WRES=0: Cin = 32 split-fp16 layers stream their weight slab per chunk (A/B timing)
static bool use_wres() {
  static const bool v = [] {
    const char* e = getenv("EBSDVAE_WRES");
    return !(e && e[0] == '0');
  }();
  return v;
}

// compute units the persistent kernels launched on stream s own: the registered count of a
// CU-masked stream (ebsdvae_stream_create_cus), else the current device's (cached per device id)
static int cu_count(hipStream_t s) {
  if (const int n = evh::stream_cus(s)) return n;
  static int cache[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

struct X3Cfg {
  int M, TH, NT, KX, nwv;
  int NI;            // images per tile (> 1 only for the pipelined kernel on small maps)
  int wr;            // pipelined split-fp16 kernel: resident weight slabs (Cin / 8), 0 = streamed
  size_t lds;        // conv3x3_split_kernel
  size_t lds_pipe;   // conv3x3_pipe_kernel (padded weight buffers); 0 = does not fit
};

// NP = 2: Cout 128 -> 8 waves x M 256; Cout 64 / 32 -> 4 waves x M 256 (2 blocks / CU).
// NP = 3: the 3-piece weight slab is 1.5x larger, so every Cout runs 8 waves (M 256 for
// Cout 128, M 512 otherwise) with one block per CU.
// NP_F16 (forward only, pipelined kernel only) takes the NP = 3 geometry with 2-piece slabs.
static bool plan_split(int H, int W, int cin, int cout, int np, X3Cfg* c) {
  if ((np != 2 && np != 3 && np != NP_F16) || cin % (2 * XCK) || !(cout == 128 || cout == 64 || cout == 32)) return false;
  if (np == NP_F16 && !use_pipe()) return false;
  // the pipelined kernel maps iterations to (image, row band, chunk) by shifts
  auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  if (!pow2(cin / XCK) || !pow2(H) || !pow2(W)) return false;
  // per-image byte ranges of the buffer descriptors (sources up to 2H x 2W for max-pool
  // modes, outputs and the fused reduce's y_prev windows): 32-bit
  if (!ev_buf_bytes_ok(4LL * H * W * (cin > cout ? cin : cout) * 4)) return false;
  c->M = (np != 2 && cout != 128) ? 512 : 256;
  c->NI = 1;
  c->NT = cout;
  c->nwv = (cout == 128 || np != 2) ? 8 : 4;
  if (H * W < c->M) {
    // 8x8 maps (bf16x6, 128 channels): tiles of two whole images, 128 pixels, 8 waves of
    // 64 px x 32 co; pipelined kernel only
    if (!((np == 3 || np == NP_F16) && cout == 128 && H * W == 64 && use_pipe() && use_multi_image()))
      return false;
    c->M = 128;
    c->NI = 2;
    c->TH = H;
    if (np == NP_F16 && use_small_one_image()) {
      // split-fp16: one image per block and 4 waves of 64 px x 32 co, so that B = 256 gives
      // 256 blocks (two-image tiles fill only half the CUs)
      c->M = 64;
      c->NI = 1;
      c->nwv = 4;
    }
  } else {
    if (W > c->M || c->M % W) return false;
    c->TH = c->M / W;
    if (H % c->TH) return false;
  }
  const int pixI = (c->TH + 2) * (W + 2);
  const int pix = c->NI * pixI;
  const int tpg = (c->nwv / c->NI) * 64;   // threads staging one image's halo
  // pipelined kernel: interior columns only; the non-persistent kernel stages whole halo rows
  c->KX = use_pipe() ? ((c->TH + 2) * W * 2 + tpg - 1) / tpg : (pixI * 2 + tpg - 1) / tpg;
  // the item count each dispatch_split instantiation is compiled for
  const int kxmax = np == 2 ? (cout == 128 ? 2 : (cout == 64 ? 5 : 7))
                            : (np == NP_F16 ? (cout == 128 ? 2 : (cout == 64 ? 3 : 4))
                                            : (cout == 128 ? 2 : (cout == 64 ? 4 : 5)));
  if (c->KX > kxmax) return false;
  const int wslab = XTAPS * npc(np) * cout * 16;
  c->lds = 2 * (size_t)wslab + 2 * (size_t)(pix + 1) * XPS;
  c->lds_pipe = 2 * (size_t)pipe_dma_per(wslab, c->nwv) * c->nwv * 1024 + 2 * (size_t)(pix + 1) * XPS;
  if (c->lds_pipe > 160 * 1024) c->lds_pipe = 0;
  // Cin = 32 split-fp16 layers (4 chunks): all four weight slabs stay resident in LDS when they
  // fit beside the two halo buffers (EBSDVAE_WRES=0 streams them per chunk, A/B)
  c->wr = 0;
  const size_t lds_wr = 4 * (size_t)wslab + 2 * (size_t)(pix + 1) * XPS;
  if (np == NP_F16 && cin == 4 * XCK && c->NI == 1 && use_wres() && use_pipe() && lds_wr <= 160 * 1024) {
    c->wr = 4;
    c->lds_pipe = lds_wr;
  }
  if (c->NI > 1 || np == NP_F16) return c->lds_pipe != 0;   // pipelined kernel only
  return c->lds <= 160 * 1024;
}

// Does the persistent kernel's tile split give every block whole images (t0 = blockIdx.x * tpb
// on an image boundary, tpb a multiple of the tiles per image), so that each block can run the
// InstanceNorm finalize of its own images after its last tile?  (B = 256 at 128^2: 32 tiles of
// 4 rows per image, 8192 tiles over 256 CUs -> exactly one image per block.)
// EBSDVAE_FUSE_FINALIZE=0 always takes the standalone finalize kernels (A/B, tests).
static bool pipe_owns_images(const X3Cfg& c, int B, int H, hipStream_t s) {
  static const bool on = [] {
    const char* e = getenv("EBSDVAE_FUSE_FINALIZE");
    return !(e && e[0] == '0');
  }();
  if (!on || !(c.NI > 1 || (use_pipe() && c.lds_pipe))) return false;
  const int tpi = c.NI > 1 ? 1 : H / c.TH;
  const int ntiles = ((B + c.NI - 1) / c.NI) * tpi;
  const int ncu = cu_count(s);
  const int tpb = (ntiles + ncu - 1) / ncu;
  return tpb % tpi == 0;
}

// ACT_FIRST: the two x tiles and the tap table behind the halo buffers
static size_t first_lds_extra(int TH, int W) {
  return (2 * (size_t)(TH + 4) * (W + 2) + FIRST_WTAB) * sizeof(float);
}

template <int NP, int NWV, int WM, int MF, int NF, int KX, int MODE, int FP, int NI, int WR = 0>
static void launch_x3_1(const X3Cfg& c, const float* src, const float* st, const void* wp,
                        const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                        int cin, hipStream_t s, const InBwdFuse& f) {
  const int ntiles = ((B + NI - 1) / NI) * (H / c.TH);
  if (NI > 1 || (use_pipe() && c.lds_pipe)) {
    auto k = conv3x3_pipe_kernel<NP, NWV, WM, MF, NF, KX, MODE, FP, NI, WR>;
    static bool once = false;
    if (!once) {
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      once = true;
    }
    // one block per CU, each owning a contiguous run of tiles
    const int ncu = cu_count(s);
    const int tpb = (ntiles + ncu - 1) / ncu;
    const int nblk = (ntiles + tpb - 1) / tpb;
    const size_t lds = c.lds_pipe + (MODE == ACT_FIRST ? first_lds_extra(c.TH, W) : 0);
    hipLaunchKernelGGL(k, dim3(nblk), dim3(NWV * 64), lds, s, src, (const float2*)st,
                       (const char*)wp, bias, y, (float2*)part, aout, B, H, W, cin, c.TH, tpb, f.yprev,
                       f.stprev, f.part, f.ypool, f.gmax, f.gmT, f.st_out, f.bst_out, f.inv_hw, f.w0,
                       f.b0);
    return;
  }
  if constexpr (NI == 1 && FP != FP_POOLOUT && NP != NP_F16) {
    auto k = conv3x3_split_kernel<NP, NWV, WM, MF, NF, KX, MODE, FP>;
    static bool once = false;
    if (!once) {
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      once = true;
    }
    hipLaunchKernelGGL(k, dim3(ntiles), dim3(NWV * 64), c.lds, s, src, (const float2*)st,
                       (const char*)wp, bias, y, (float2*)part, aout, B, H, W, cin, c.TH, f.yprev,
                       f.stprev, f.part);
  }
}

template <int NP, int NWV, int WM, int MF, int NF, int KX, int NI = 1, int WR = 0>
static void launch_x3(const X3Cfg& c, const float* src, const float* st, int mode, const void* wp,
                      const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                      int cin, hipStream_t s, int pmode, const InBwdFuse& f) {
  if (pmode >= 0) {
    switch (pmode) {
      case P_ID: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, P_ID, NI, WR>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
      case P_POOL: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, P_POOL, NI, WR>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
      case P_UPSUM:
        if constexpr (NI == 1)
          launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, FP_UPSUM, NI, WR>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f);
        break;
      default: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, P_UP, NI, WR>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
    }
    return;
  }
  if constexpr (NI == 1) {
    if (f.ypool) {   // producer of a max-pooled layer (ebsdvae_conv3x3_fwd_split_pooled)
      launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM, FP_POOLOUT, NI, WR>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f);
      return;
    }
  }
  switch (mode) {
    case ACT_RAW: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, FP_NONE, NI, WR>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_NORM: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM, FP_NONE, NI, WR>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_NORM_POOL: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM_POOL, FP_NONE, NI, 0>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_UP: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_UP, FP_NONE, NI, WR>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    default: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM_UP, FP_NONE, NI, WR>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
  }
}

static void dispatch_split(const X3Cfg& c, int np, const float* src, const float* st, int mode,
                           const void* wp, const float* bias, float* y, float* part, float* aout,
                           int B, int H, int W, int cin, int cout, hipStream_t s, int pmode,
                           const InBwdFuse& f) {
  if (np == 2) {
    if (cout == 128)
      launch_x3<2, 8, 4, 2, 2, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 64)
      launch_x3<2, 4, 4, 2, 2, 5>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else
      launch_x3<2, 4, 4, 2, 1, 7>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
  } else if (np == NP_F16) {
    if (cout == 128 && c.NI > 1)   // two 8x8 images per tile
      launch_x3<NP_F16, 8, 2, 2, 1, 1, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 128 && c.M == 64)   // one 8x8 image per tile, 4 waves
      launch_x3<NP_F16, 4, 1, 2, 1, 1>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 128)
      launch_x3<NP_F16, 8, 4, 2, 2, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 64 && c.wr)   // Cin = 32: weight slabs resident
      launch_x3<NP_F16, 8, 8, 2, 2, 3, 1, 4>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 64)
      launch_x3<NP_F16, 8, 8, 2, 2, 3>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (c.KX <= 3 && c.wr)
      launch_x3<NP_F16, 8, 8, 2, 1, 3, 1, 4>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (c.KX <= 3)
      launch_x3<NP_F16, 8, 8, 2, 1, 3>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (c.wr)   // 256-wide maps: two-row tiles, four items per thread
      launch_x3<NP_F16, 8, 8, 2, 1, 4, 1, 4>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else
      launch_x3<NP_F16, 8, 8, 2, 1, 4>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
  } else {
    if (cout == 128 && c.NI > 1)   // two 8x8 images per tile: 2 x 4 waves of 64 px x 32 co
      launch_x3<3, 8, 2, 2, 1, 1, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 128)
      launch_x3<3, 8, 4, 2, 2, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 64)
      launch_x3<3, 8, 8, 2, 2, 4>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else
      launch_x3<3, 8, 8, 2, 1, 5>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
  }
}

}  // namespace ev

using namespace ev;

#ifdef EV_PIPE_TRACE
extern "C" int ebsdvae_debug_pipe_trace(void* host, size_t bytes) {
  if (bytes > sizeof(ev_pipe_trace)) bytes = sizeof(ev_pipe_trace);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ev_pipe_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int ebsdvae_conv3x3_split_supported(int H, int W, int cin, int cout, int pieces) {
  X3Cfg c;
  return plan_split(H, W, cin, cout, pieces, &c) ? 1 : 0;
}

extern "C" int ebsdvae_conv3x3_split_stat_tiles(int H, int W, int cout) {
  (void)cout;
  if (!ev_dim_ok(H) || !ev_dim_ok(W)) return -1;
  return (H * W) / 64;   // every split configuration writes one statistics slot per 64 pixels
}

extern "C" size_t ebsdvae_pack_split_bytes(int cin, int cout, int pieces) {
  if (cin <= 0 || cout <= 0 || !(pieces == 2 || pieces == 3 || pieces == NP_F16)) return 0;
  return (size_t)(cin / XCK) * XTAPS * npc(pieces) * cout * XCK * 2 +
         (pieces == NP_F16 ? kF16PackTrailer : 0);
}

extern "C" int ebsdvae_pack_conv_weights_split(const ebsdvae_pack_desc* descs, int n, int pieces,
                                               ebsdvae_stream_t stream) {
  EV_REQUIRE(descs && n > 0 && n <= EBSDVAE_MAX_PACK, "pack_conv_weights_split: n=%d out of range", n);
  EV_REQUIRE(pieces == 2 || pieces == 3 || pieces == NP_F16,
             "pack_conv_weights_split: pieces=%d (2, 3 or %d)", pieces, NP_F16);
  PackBatch pb;
  int maxn = 0;
  for (int i = 0; i < n; ++i) {
    const ebsdvae_pack_desc& q = descs[i];
    const int ci_ = q.for_dgrad ? q.cout : q.cin;
    EV_REQUIRE(q.src && q.dst && q.cin > 0 && q.cout > 0 && (q.kind == 0 || q.kind == 1) && ci_ % XCK == 0,
               "pack_conv_weights_split: bad descriptor %d", i);
    pb.d[i] = q;
    const int e = (ci_ / XCK) * XTAPS * (q.for_dgrad ? q.cin : q.cout) * XCK;
    if (e > maxn) maxn = e;
  }
  int bx = (maxn + 255) / 256;
  if (bx > 64) bx = 64;
  if (pieces == NP_F16)
    hipLaunchKernelGGL(pack_wmax_kernel, dim3(kF16MaxParts, n), dim3(256), 0, (hipStream_t)stream, pb);
  hipLaunchKernelGGL(pack_split_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, pb, pieces);
  return evh::check_launch("pack_conv_weights_split");
}

extern "C" int ebsdvae_conv3x3_fwd_split(const float* src, const float* src_stats, int src_mode,
                                         const void* wpack, const float* bias, float* y,
                                         float* stat_part, float* act_out, int B, int H, int W,
                                         int cin, int cout, int pieces, ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(src && wpack && y && B > 0, "conv3x3_fwd_split: null pointer or empty batch");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4, "conv3x3_fwd_split: bad src_mode %d", src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats,
             "conv3x3_fwd_split: NORM modes need src_stats");
  EV_REQUIRE(plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_fwd_split: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W, cin, cout,
             pieces);
  dispatch_split(c, pieces, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W,
                 cin, cout, (hipStream_t)stream, -1, InBwdFuse());
  return evh::check_launch("conv3x3_fwd_split");
}

extern "C" int ebsdvae_conv3x3_split_pool_ok(int H, int W, int cin, int cout, int pieces) {
  X3Cfg c;
  return (plan_split(H, W, cin, cout, pieces, &c) && use_pipe() && c.lds_pipe && c.NI == 1 &&
          c.TH % 2 == 0 && W >= 16 && (W & (W - 1)) == 0) ? 1 : 0;
}

extern "C" int ebsdvae_conv3x3_fwd_split_pooled(const float* src, const float* src_stats,
                                                int src_mode, const void* wpack, const float* bias,
                                                float* y, float* ypool, float* stat_part, int B,
                                                int H, int W, int cin, int cout, int pieces,
                                                ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(src && src_stats && wpack && y && ypool && stat_part && B > 0,
             "conv3x3_fwd_split_pooled: null pointer or empty batch");
  EV_REQUIRE(src_mode == ACT_NORM, "conv3x3_fwd_split_pooled: src_mode %d (ACT_NORM only)", src_mode);
  EV_REQUIRE(ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, pieces) && plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_fwd_split_pooled: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W,
             cin, cout, pieces);
  InBwdFuse f;
  f.ypool = ypool;
  dispatch_split(c, pieces, src, src_stats, src_mode, wpack, bias, y, stat_part, nullptr, B, H, W,
                 cin, cout, (hipStream_t)stream, -1, f);
  return evh::check_launch("conv3x3_fwd_split_pooled");
}

extern "C" int ebsdvae_conv3x3_dgrad_inbwd_split(const float* g, const void* wpack, float* gin,
                                                 const float* y_prev, const float* st_prev,
                                                 int pmode, double* part, int B, int H, int W,
                                                 int cin, int cout, int pieces,
                                                 ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(g && wpack && gin && B > 0, "conv3x3_dgrad_inbwd_split: null pointer or empty batch");
  EV_REQUIRE(pieces != NP_F16, "conv3x3_dgrad_inbwd_split: fp16 pieces need the gradient scale "
             "(ebsdvae_conv3x3_dgrad_inbwd_f16)");
  EV_REQUIRE(pmode >= -1 && pmode <= P_UPSUM, "conv3x3_dgrad_inbwd_split: bad pmode %d", pmode);
  EV_REQUIRE(pmode != P_UPSUM || ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, pieces),
             "conv3x3_dgrad_inbwd_split: summed upsample adjoint unsupported for H=%d W=%d", H, W);
  EV_REQUIRE(pmode < 0 || (y_prev && st_prev && part && (W & (W - 1)) == 0),
             "conv3x3_dgrad_inbwd_split: fused reduce needs y_prev, st_prev, part and W = 2^k");
  EV_REQUIRE(plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_dgrad_inbwd_split: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W,
             cin, cout, pieces);
  InBwdFuse f;
  f.yprev = y_prev;
  f.stprev = (const float2*)st_prev;
  f.part = (double2*)part;
  dispatch_split(c, pieces, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin,
                 cout, (hipStream_t)stream, pmode, f);
  return evh::check_launch("conv3x3_dgrad_inbwd_split");
}

extern "C" int ebsdvae_conv3x3_dgrad_inbwd_f16(const float* g, const float* gmax, int gm_tiles,
                                               const void* wpack, float* gin, const float* y_prev,
                                               const float* st_prev, int pmode, double* part, int B,
                                               int H, int W, int cin, int cout,
                                               ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(g && gmax && gm_tiles > 0 && wpack && gin && B > 0,
             "conv3x3_dgrad_inbwd_f16: null pointer, empty batch or no gradient maxima");
  EV_REQUIRE(pmode >= -1 && pmode <= P_UPSUM, "conv3x3_dgrad_inbwd_f16: bad pmode %d", pmode);
  EV_REQUIRE(pmode != P_UPSUM || ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, NP_F16),
             "conv3x3_dgrad_inbwd_f16: summed upsample adjoint unsupported for H=%d W=%d", H, W);
  EV_REQUIRE(pmode < 0 || (y_prev && st_prev && part && (W & (W - 1)) == 0),
             "conv3x3_dgrad_inbwd_f16: fused reduce needs y_prev, st_prev, part and W = 2^k");
  EV_REQUIRE(plan_split(H, W, cin, cout, NP_F16, &c),
             "conv3x3_dgrad_inbwd_f16: unsupported shape H=%d W=%d cin=%d cout=%d", H, W, cin, cout);
  InBwdFuse f;
  f.yprev = y_prev;
  f.stprev = (const float2*)st_prev;
  f.part = (double2*)part;
  f.gmax = gmax;
  f.gmT = gm_tiles;
  dispatch_split(c, NP_F16, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin,
                 cout, (hipStream_t)stream, pmode, f);
  return evh::check_launch("conv3x3_dgrad_inbwd_f16");
}

// Forward split conv + its InstanceNorm statistics st (B, cout) {mean, rstd}: finalized by the
// conv's own blocks when they own whole images (pipe_owns_images), otherwise by the standalone
// finalize kernel after it; bit-identical either way.  ypool != NULL: the pooled producer form.
extern "C" int ebsdvae_conv3x3_fwd_split_st(const float* src, const float* src_stats, int src_mode,
                                            const void* wpack, const float* bias, float* y,
                                            float* ypool, float* stat_part, float* st, int B,
                                            int H, int W, int cin, int cout, int pieces,
                                            ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(src && wpack && (y || ypool) && stat_part && st && B > 0,
             "conv3x3_fwd_split_st: null pointer or empty batch");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4, "conv3x3_fwd_split_st: bad src_mode %d", src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats,
             "conv3x3_fwd_split_st: NORM modes need src_stats");
  EV_REQUIRE(!ypool || (src_mode == ACT_NORM && ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, pieces)),
             "conv3x3_fwd_split_st: pooled output unsupported for H=%d W=%d src_mode=%d", H, W, src_mode);
  EV_REQUIRE(plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_fwd_split_st: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W, cin,
             cout, pieces);
  const bool fused = pipe_owns_images(c, B, H, (hipStream_t)stream);
  InBwdFuse f;
  f.ypool = ypool;
  if (fused) f.st_out = (float2*)st;
  dispatch_split(c, pieces, src, src_stats, src_mode, wpack, bias, y, stat_part, nullptr, B, H, W,
                 cin, cout, (hipStream_t)stream, -1, f);
  if (int rc = evh::check_launch("conv3x3_fwd_split_st")) return rc;
  if (fused) return 0;
  const int T = ebsdvae_conv3x3_split_stat_tiles(H, W, cout);
  return ebsdvae_in_stats_finalize(stat_part, st, B, cout, T, (H * W) / T, stream);
}

// ebsdvae_conv3x3_dgrad_inbwd_f16 with a fused reduce (pmode >= 0) that also returns the
// previous block's finalized InstanceNorm-backward statistics bst (B, cin) over prev_hw pixels
// (what ebsdvae_in_bwd_finalize makes of part), in-kernel where pipe_owns_images allows.
extern "C" int ebsdvae_conv3x3_dgrad_inbwd_f16_bst(const float* g, const float* gmax, int gm_tiles,
                                                   const void* wpack, float* gin, const float* y_prev,
                                                   const float* st_prev, int pmode, double* part,
                                                   float* bst, int prev_hw, int B, int H, int W,
                                                   int cin, int cout, ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(g && gmax && gm_tiles > 0 && wpack && gin && B > 0,
             "conv3x3_dgrad_inbwd_f16_bst: null pointer, empty batch or no gradient maxima");
  EV_REQUIRE(pmode >= 0 && pmode <= P_UPSUM && y_prev && st_prev && part && bst && prev_hw > 0 &&
                 (W & (W - 1)) == 0,
             "conv3x3_dgrad_inbwd_f16_bst: fused reduce needs pmode >= 0, y_prev, st_prev, part, bst, "
             "prev_hw and W = 2^k");
  EV_REQUIRE(pmode != P_UPSUM || ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, NP_F16),
             "conv3x3_dgrad_inbwd_f16_bst: summed upsample adjoint unsupported for H=%d W=%d", H, W);
  EV_REQUIRE(plan_split(H, W, cin, cout, NP_F16, &c),
             "conv3x3_dgrad_inbwd_f16_bst: unsupported shape H=%d W=%d cin=%d cout=%d", H, W, cin, cout);
  const bool fused = pipe_owns_images(c, B, H, (hipStream_t)stream);
  InBwdFuse f;
  f.yprev = y_prev;
  f.stprev = (const float2*)st_prev;
  f.part = (double2*)part;
  f.gmax = gmax;
  f.gmT = gm_tiles;
  if (fused) {
    f.bst_out = (float2*)bst;
    f.inv_hw = 1.0 / (double)prev_hw;
  }
  dispatch_split(c, NP_F16, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin,
                 cout, (hipStream_t)stream, pmode, f);
  if (int rc = evh::check_launch("conv3x3_dgrad_inbwd_f16_bst")) return rc;
  if (fused) return 0;
  // (cin, cout) are the conv's: gin and the previous block have cout channels
  return ebsdvae_in_bwd_finalize(part, bst, B, cout, ebsdvae_conv3x3_split_stat_tiles(H, W, cout), prev_hw,
                                 stream);
}

// The second block's forward with the first block recomputed from x (ACT_FIRST staging):
// encoder.1 of latice/model.py:111 reading lrelu(IN(conv(x, w0) + b0)) without y0.
extern "C" int ebsdvae_conv3x3_fwd_split_first_ok(int H, int W, int cin, int cout, int pieces) {
  X3Cfg c;
  if (pieces != NP_F16 || cin != 4 * XCK || cout != 32 || !plan_split(H, W, cin, cout, pieces, &c))
    return 0;
  if (!(use_pipe() && c.wr && c.NI == 1 && (c.KX == 3 || c.KX == 4))) return 0;
  if ((size_t)(c.TH + 4) * (W + 2) > 4 * (size_t)c.nwv * 64) return 0;   // XTN x-tile registers
  return c.lds_pipe + first_lds_extra(c.TH, W) <= 160 * 1024 ? 1 : 0;
}

extern "C" int ebsdvae_conv3x3_fwd_split_first(const float* x, const float* st0, const float* w0,
                                               const float* b0, const void* wpack, const float* bias,
                                               float* y, float* ypool, float* stat_part, float* st,
                                               int B, int H, int W, int cin, int cout, int pieces,
                                               ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(x && st0 && w0 && wpack && (y || ypool) && stat_part && st && B > 0,
             "conv3x3_fwd_split_first: null pointer or empty batch");
  EV_REQUIRE(ebsdvae_conv3x3_fwd_split_first_ok(H, W, cin, cout, pieces) &&
                 plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_fwd_split_first: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W, cin,
             cout, pieces);
  EV_REQUIRE(!ypool || ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, pieces),
             "conv3x3_fwd_split_first: pooled output unsupported for H=%d W=%d", H, W);
  hipStream_t s = (hipStream_t)stream;
  const bool fused = pipe_owns_images(c, B, H, s);
  InBwdFuse f;
  f.ypool = ypool;
  f.w0 = w0;
  f.b0 = b0;
  if (fused) f.st_out = (float2*)st;
  if (ypool) {
    if (c.KX == 3)
      launch_x3_1<NP_F16, 8, 8, 2, 1, 3, ACT_FIRST, FP_POOLOUT, 1, 4>(c, x, st0, wpack, bias, y, stat_part, nullptr, B, H, W, cin, s, f);
    else
      launch_x3_1<NP_F16, 8, 8, 2, 1, 4, ACT_FIRST, FP_POOLOUT, 1, 4>(c, x, st0, wpack, bias, y, stat_part, nullptr, B, H, W, cin, s, f);
  } else {
    if (c.KX == 3)
      launch_x3_1<NP_F16, 8, 8, 2, 1, 3, ACT_FIRST, FP_NONE, 1, 4>(c, x, st0, wpack, bias, y, stat_part, nullptr, B, H, W, cin, s, f);
    else
      launch_x3_1<NP_F16, 8, 8, 2, 1, 4, ACT_FIRST, FP_NONE, 1, 4>(c, x, st0, wpack, bias, y, stat_part, nullptr, B, H, W, cin, s, f);
  }
  if (int rc = evh::check_launch("conv3x3_fwd_split_first")) return rc;
  if (fused) return 0;
  const int T = ebsdvae_conv3x3_split_stat_tiles(H, W, cout);
  return ebsdvae_in_stats_finalize(stat_part, st, B, cout, T, (H * W) / T, stream);
}
