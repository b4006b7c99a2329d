/*
 * ebsdvae.h — C ABI of the MI355X-native VAE hot path (libebsdvae.so, gfx950).
 *
 * The reference (poyentung/ebsd-vae, package `latice`) has NO native boundary: its hot
 * path is `VariationalAutoEncoderRawData.forward` (latice/model.py:40-66, built at
 * :90-150) plus `VAELoss.compute_loss` (latice/lightning_module.py:122-156), executed as
 * ATen ops.  Each entry point below replaces the ATen work of one of those source lines;
 * the citation after each declaration names it.  The Python layer
 * (ebsd-vae_amd/latice/_native.py) binds these with ctypes, exactly as INTEGRATION.md
 * shows.
 *
 * Contract (every function):
 *  - all tensor arguments are DEVICE pointers to fp32 (unless noted), NHWC for
 *    activations; `stream` is a hipStream_t (NULL = default stream);
 *  - the library never allocates, frees or synchronises; scratch buffers are sized with
 *    the *_size / *_count queries and owned by the caller;
 *  - return 0 on success; nonzero on invalid shape or launch failure, with a message in
 *    ebsdvae_last_error() (thread-local);
 *  - stateless: safe to call concurrently on different streams; capturable into hipGraphs.
 *
 * "act source" arguments (src, src_stats, src_mode) describe how a consumer reads its
 * input: mode 0 RAW, 1 NORM = lrelu((src-mean)*rstd), 2 NORM_POOL (2x2 max of NORM, src
 * at 2x resolution), 3 UP (nearest x2 of src at half resolution), 4 NORM_UP.
 * src_stats is float2 {mean, rstd} per (b, c) (NULL for RAW/UP).
 */
#ifndef EBSDVAE_H_
#define EBSDVAE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* ebsdvae_stream_t; /* hipStream_t */

const char* ebsdvae_last_error(void);
/* ABI version of this header; ebsdvae_version() returns the library's.  Bumped on every
 * incompatible signature change (2: ebsdvae_heads_fwd / _bwd / ebsdvae_latent_mu take a
 * caller-owned `work` scratch pointer).  Callers must check it before the first call. */
#define EBSDVAE_ABI_VERSION 2
int ebsdvae_version(void);

/* ---- stream ordering ------------------------------------------------------------------
 * `waiter` waits for the work enqueued on `signaler` so far (an event with the default
 * system-scope release; EBSDVAE_FORK_DEVICE_SCOPE=1: device scope, as through round 5).
 * Used for the weight-gradient side stream's fork / join (latice/engine.py); capturable. */
int ebsdvae_stream_wait(ebsdvae_stream_t waiter, ebsdvae_stream_t signaler);
/* Kernel-attached fork (no record packet on the signaler): arm, launch the InstanceNorm-backward
 * apply (ebsdvae_in_bwd_apply[_max]) on `signaler`, then ebsdvae_fork_wait makes `waiter` wait
 * for that launch's completion (falls back to ebsdvae_stream_wait when nothing took the event).
 * Per host thread. */
int ebsdvae_fork_arm(ebsdvae_stream_t signaler);
int ebsdvae_fork_wait(ebsdvae_stream_t waiter, ebsdvae_stream_t signaler);
/* CU-partitioned streams (experiment): a new stream restricted to the
 * compute units of CU-mask bits [first, first + count) (count a multiple of 8; the runtime
 * spreads contiguous bits evenly over the XCDs).  The persistent conv kernels launched on it
 * size their grids by `count`.  Destroy with ebsdvae_stream_destroy_cus. */
int ebsdvae_stream_create_cus(int first, int count, ebsdvae_stream_t* out);
int ebsdvae_stream_destroy_cus(ebsdvae_stream_t stream);

/* ---- weights ------------------------------------------------------------------------
 * Pack a Conv2d (kind 0: (cout,cin,3,3), latice/model.py:95,148) or ConvTranspose2d
 * (kind 1: (cin,cout,3,3), latice/model.py:102-104) weight into the kernel layout
 * [Cin'/8][tap][8][Cout'] (one contiguous slab per 8-channel K chunk).  for_dgrad=0: the forward conv (Cin'=cin, Cout'=cout);
 * for_dgrad=1: the input-gradient conv (Cin'=cout, Cout'=cin, taps flipped). */
int ebsdvae_pack_conv_weight(const float* src, float* dst, int cin, int cout, int kind,
                             int for_dgrad, ebsdvae_stream_t stream);

/* Batched form: n <= EBSDVAE_MAX_PACK descriptors in HOST memory (passed to the kernel by
 * value), one launch for every conv weight of a step. */
#define EBSDVAE_MAX_PACK 64
typedef struct {
  const float* src; /* device */
  float* dst;       /* device */
  int cin, cout, kind, for_dgrad;
} ebsdvae_pack_desc;
int ebsdvae_pack_conv_weights(const ebsdvae_pack_desc* descs, int n, ebsdvae_stream_t stream);

/* ---- 3x3 conv, implicit GEMM on fp32 MFMA -------------------------------------------
 * y[b,h,w,co] = bias[co] + sum_{tap,ci} act(src)[b,h+dh,w+dw,ci] * wpack[tap][ci][co]
 * (zero padding 1).  Replaces nn.Conv2d / nn.ConvTranspose2d forward
 * (latice/model.py:95,102-104) and, with a for_dgrad pack and RAW source, their input
 * gradients.  If stat_part != NULL, also writes per-tile InstanceNorm partials
 * {mean, M2} per (b, tile, co) (count ebsdvae_conv3x3_stat_tiles per image).  If
 * act_out != NULL, also writes the conv's logical input act(src) as (B,H,W,cin) NHWC (used
 * for max-pool-fed layers, whose weight gradient then reads the 4x smaller pooled tensor).
 * cin in {1} U {8k}, cout in {32, 64, 128}; W <= tile width (128x128 and 256x256 nets).
 * bias may be NULL.  wpack layout: [cin/8][tap][8][cout] (ebsdvae_pack_conv_weight). */
int ebsdvae_conv3x3_fwd(const float* src, const float* src_stats, int src_mode,
                        const float* wpack, const float* bias, float* y, float* stat_part,
                        float* act_out, int B, int H, int W, int cin, int cout,
                        ebsdvae_stream_t stream);
int ebsdvae_conv3x3_stat_tiles(int H, int W, int cout);

/* Input gradient of a conv (ebsdvae_conv3x3_fwd with a for_dgrad pack and RAW source:
 * g = d loss / d a_prev at (B,H,W,cout) NHWC) fused with the reduce pass of the
 * PREVIOUS block's InstanceNorm backward (ebsdvae_in_bwd_reduce(g, pmode, y_prev,
 * st_prev, ...)).  a_prev = pmode(lrelu(IN(y_prev))); y_prev is (B,2H,2W,cout) for P_POOL,
 * (B,H/2,W/2,cout) for P_UP, (B,H,W,cout) for P_ID.  part receives double2
 * {sum h, sum h*xhat} per (b, tile, c) with ebsdvae_conv3x3_stat_tiles(H,W,cout) tiles
 * per image; ebsdvae_in_bwd_finalize(part, ..., tiles, HW of y_prev) turns them into the
 * apply-pass statistics.  gin receives h = g * lrelu'(xhat), xhat that of the y_prev pixel g
 * routes to (the first 2x2 argmax for P_POOL, the parent for P_UP): the operand of
 * ebsdvae_in_bwd_happly / _first_happly_wgrad*, which need no LeakyReLU branch of their own.
 * Every fused input-gradient entry point below (pmode >= 0) writes h the same way.
 * Replaces autograd's conv input gradient plus the first half of the InstanceNorm backward
 * (latice/model.py:95-97,102-106).  W must be a power of two. */
int ebsdvae_conv3x3_dgrad_inbwd(const float* g, const float* wpack, float* gin,
                                const float* y_prev, const float* st_prev, int pmode,
                                double* part, int B, int H, int W, int cin, int cout,
                                ebsdvae_stream_t stream);

/* 3x3 conv with a single output channel (the final nn.Conv2d(32,1), latice/model.py:148):
 * out[b,h,w] = bias + sum act(src)*w[ci][tap'] with tap' = flip ? 8-tap : tap.
 * w is (1,cin,3,3) contiguous (== (cin,1,3,3)).  With flip=1, RAW source and
 * w = encoder.0 weight it is the input gradient of the first conv. bias may be NULL. */
/* The first conv nn.Conv2d(1, C, 3, 1, 1) (latice/model.py:110), C == 32, on the VALU:
 * y (B,H,W,C) NHWC = conv(x (B,1,H,W), w0 (C,1,3,3)) + b0 (b0 may be NULL), and its
 * InstanceNorm partials part[b][t][c] = {mean, M2} over row band t of n = H*W/T pixels,
 * T = ebsdvae_conv_first_stat_tiles(H, W) (-1: shape unsupported; W must divide 512), for
 * ebsdvae_in_stats_finalize.  Its arithmetic is the fixed fma chain that
 * ebsdvae_in_bwd_first_apply_wgrad_rc and ebsdvae_conv3x3_fwd_split_first recompute y with.
 * y may be NULL: the statistics only (inference, where the next conv recomputes y from x). */
int ebsdvae_conv_first_stat_tiles(int H, int W);
/* The InstanceNorm statistics st (B, C) {mean, rstd} of y0 = the first conv of x (C == 32)
 * without computing y0: from the 9 shifted means and the 45 shifted second moments of x per
 * image, in double (mean_c = b_c + sum_t w_ct m_t, var_c = sum_tt' w_ct w_ct' cov_tt').  The
 * inference path's first conv (y0 is recomputed by ebsdvae_conv3x3_fwd_split_first).  Needs W
 * dividing 256 and H % 32 == 0. */
int ebsdvae_conv_first_stats(const float* x, const float* w0, const float* b0, float* st, int B,
                             int H, int W, int C, ebsdvae_stream_t stream);

int ebsdvae_conv_first_fwd(const float* x, const float* w0, const float* b0, float* y,
                           float* part, int B, int H, int W, int C, ebsdvae_stream_t stream);
int ebsdvae_conv3x3_cout1_fwd(const float* src, const float* src_stats, int src_mode,
                              const float* w, const float* bias, float* out, int flip,
                              int B, int H, int W, int cin, ebsdvae_stream_t stream);
/* input gradient of the cout=1 conv: gin[b,h,w,ci] = sum_tap g[b,h-dh,w-dw] * w[ci][tap] */
int ebsdvae_conv3x3_cout1_dgrad(const float* g, const float* w, float* gin, int B, int H,
                                int W, int cin, ebsdvae_stream_t stream);

/* ---- split-bf16 conv: same semantics as ebsdvae_conv3x3_fwd / _dgrad_inbwd ---------------
 * Each fp32 operand is carried as `pieces` bf16 pieces (x0 = bf16(x), x1 = bf16(x - x0),
 * x2 = bf16(x - x0 - x1)) and every product keeps the terms of total order < pieces, on
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation:
 *   pieces = 2 ("bf16x3", 3 MFMAs, ~2^-16.5 relative error per product);
 *   pieces = 3 ("bf16x6", 6 MFMAs, ~2^-25: fp32 grade);
 *   pieces = EBSDVAE_PIECES_F16 ("f16x3": two fp16 pieces x0 = f16(x), x1 = f16(x - x0) on
 *     v_mfma_f32_32x32x16_f16, 3 MFMAs, ~2^-22.5 per product; the pack holds w * 2^k with one
 *     power of two per layer, max |w| 2^k in [2^11, 2^12), k in a trailer that
 *     ebsdvae_pack_split_bytes includes (int32 k in its 16-byte head, then 64 partial maxima
 *     of |w| it is reduced from), so any weight magnitude keeps fp16's full precision).
 * Weights use the split pack ([cin'/8][tap 0..9][piece][cout'][8] bf16,
 * ebsdvae_pack_split_bytes bytes).  Shapes: ebsdvae_conv3x3_split_supported; InstanceNorm
 * partials use ebsdvae_conv3x3_split_stat_tiles tiles per image.  pmode = -1 in
 * ebsdvae_conv3x3_dgrad_inbwd_split is a plain input gradient (y_prev/st_prev/part unused). */
#define EBSDVAE_PIECES_F16 16
int ebsdvae_conv3x3_split_supported(int H, int W, int cin, int cout, int pieces);
int ebsdvae_conv3x3_split_stat_tiles(int H, int W, int cout);
size_t ebsdvae_pack_split_bytes(int cin, int cout, int pieces);
int ebsdvae_pack_conv_weights_split(const ebsdvae_pack_desc* descs, int n, int pieces,
                                    ebsdvae_stream_t stream);
int ebsdvae_conv3x3_fwd_split(const float* src, const float* src_stats, int src_mode,
                              const void* wpack, const float* bias, float* y, float* stat_part,
                              float* act_out, int B, int H, int W, int cin, int cout, int pieces,
                              ebsdvae_stream_t stream);
/* Forward of a layer whose output the next layer max-pools (latice/model.py:111-112, 114-115,
 * 117-118, 120-121: building_blocks then nn.MaxPool2d(2, 2)): as ebsdvae_conv3x3_fwd_split
 * (src_mode ACT_NORM) and also writes ypool = the 2x2 max of the raw output y, (B, H/2, W/2,
 * cout) NHWC.  Because InstanceNorm's scale is positive and LeakyReLU is increasing,
 * maxpool(lrelu(IN(y))) == lrelu(IN(ypool)) exactly, so the next conv reads ypool in ACT_NORM
 * mode with y's statistics instead of pooling y itself.  The statistics partials group pixels
 * differently from ebsdvae_conv3x3_fwd_split (row pairs), so they can differ in the last bits.
 * ebsdvae_conv3x3_split_pool_ok: 1 if the shape is supported. */
int ebsdvae_conv3x3_split_pool_ok(int H, int W, int cin, int cout, int pieces);
int ebsdvae_conv3x3_fwd_split_pooled(const float* src, const float* src_stats, int src_mode,
                                     const void* wpack, const float* bias, float* y, float* ypool,
                                     float* stat_part, int B, int H, int W, int cin, int cout,
                                     int pieces, ebsdvae_stream_t stream);
/* pmode 3 (P_UPSUM) in ebsdvae_conv3x3_dgrad_inbwd_split: as P_UP (the block feeding this
 * conv was nearest-upsampled, latice/model.py:134-146), but gin receives the 2x2 window sums
 * of the input gradient, (B, H/2, W/2, cout) -- the gradient w.r.t. the pre-upsample
 * activation -- and ebsdvae_in_bwd_apply then takes it with pmode 0.  Shapes:
 * ebsdvae_conv3x3_split_pool_ok(H, W, cin, cout, pieces). */
int ebsdvae_conv3x3_dgrad_inbwd_split(const float* g, const void* wpack, float* gin,
                                      const float* y_prev, const float* st_prev, int pmode,
                                      double* part, int B, int H, int W, int cin, int cout,
                                      int pieces, ebsdvae_stream_t stream);
/* Input gradient on split-fp16 pieces (pieces = EBSDVAE_PIECES_F16, wpack from
 * ebsdvae_pack_conv_weights_split with for_dgrad = 1): as ebsdvae_conv3x3_dgrad_inbwd_split,
 * but g is scaled per image by 2^k (k such that max|g[b]| * 2^k lies in [2^11, 2^12)) before
 * the fp16 split and unscaled in the epilogue, so gradients of any magnitude keep fp16's 22
 * significand bits.  gmax: (B, gm_tiles) per-tile maxima of |g| from
 * ebsdvae_in_bwd_apply_max (gm_tiles = ebsdvae_in_bwd_apply_tiles). */
int ebsdvae_conv3x3_dgrad_inbwd_f16(const float* g, const float* gmax, int gm_tiles,
                                    const void* wpack, float* gin, const float* y_prev,
                                    const float* st_prev, int pmode, double* part, int B, int H,
                                    int W, int cin, int cout, ebsdvae_stream_t stream);
/* The same launches with the InstanceNorm finalize folded in (one launch where the
 * persistent kernel's blocks each own whole images, e.g. B = 256 at 128x128 -- then every
 * block finalizes its own images after its last tile -- else the conv followed by the
 * standalone finalize; bit-identical either way, EBSDVAE_FUSE_FINALIZE=0 forces the latter):
 *   _fwd_split_st: ebsdvae_conv3x3_fwd_split (ypool = NULL) or _fwd_split_pooled (ypool set),
 *     then ebsdvae_in_stats_finalize(stat_part, st, B, cout, tiles, H*W/tiles) -> st (B, cout)
 *     {mean, rstd}; with ypool set, y may be NULL (inference: the full-resolution output is
 *     then not written, st and ypool are unchanged);
 *   _dgrad_inbwd_f16_bst: ebsdvae_conv3x3_dgrad_inbwd_f16 with pmode >= 0, then
 *     ebsdvae_in_bwd_finalize(part, bst, B, cout, tiles, prev_hw) -> bst (B, cout), with
 *     (cin, cout) the channels of g and gin as in ebsdvae_conv3x3_dgrad_inbwd_f16 and prev_hw
 *     the H*W of y_prev.
 * Replace the conv + finalize pairs of the training step (latice/model.py:95-97 forward,
 * their autograd backward). */
int ebsdvae_conv3x3_fwd_split_st(const float* src, const float* src_stats, int src_mode,
                                 const void* wpack, const float* bias, float* y, float* ypool,
                                 float* stat_part, float* st, int B, int H, int W, int cin,
                                 int cout, int pieces, ebsdvae_stream_t stream);
/* The second conv block's forward (latice/model.py:111, encoder.1) with its input -- the
 * first block's activation lrelu(IN(y0)), y0 = conv(x, w0) + b0 -- recomputed from x while the
 * halo is staged, so y0 is never read (inference: never written either):
 *   x (B,1,H,W), st0 (B, cin) {mean, rstd} of y0 (ebsdvae_conv_first_fwd with y = NULL +
 *   ebsdvae_in_stats_finalize), w0 (cin,1,3,3), b0 (cin) or NULL;
 *   the rest as ebsdvae_conv3x3_fwd_split_st with src_mode = ACT_NORM on y0.
 * Each staged value is the first conv's own fma chain (ebsdvae_conv_first_fwd) followed by the
 * same normalisation, so y, ypool and st are bit-identical to the two-launch form.  Needs
 * pieces = EBSDVAE_PIECES_F16 and cin = 32 (the split kernel's resident-weight form):
 * ebsdvae_conv3x3_fwd_split_first_ok returns 1 for a supported shape, 0 otherwise. */
int ebsdvae_conv3x3_fwd_split_first_ok(int H, int W, int cin, int cout, int pieces);
int ebsdvae_conv3x3_fwd_split_first(const float* x, const float* st0, const float* w0,
                                    const float* b0, const void* wpack, const float* bias,
                                    float* y, float* ypool, float* stat_part, float* st, int B,
                                    int H, int W, int cin, int cout, int pieces,
                                    ebsdvae_stream_t stream);
int ebsdvae_conv3x3_dgrad_inbwd_f16_bst(const float* g, const float* gmax, int gm_tiles,
                                        const void* wpack, float* gin, const float* y_prev,
                                        const float* st_prev, int pmode, double* part, float* bst,
                                        int prev_hw, int B, int H, int W, int cin, int cout,
                                        ebsdvae_stream_t stream);

/* ---- weight gradients (deterministic two-level reduction) -----------------------------
 * Partial dW[co][ci][tap] and db[co] over pixel slices; then ebsdvae_wgrad_reduce sums
 * the slices in fixed order into the parameter-gradient layout of `kind` (0 conv,
 * 1 convT).  Replaces autograd's convolution_backward weight/bias outputs.
 * gy is the conv-output gradient (NHWC, cout channels); src/act as in the forward, except
 * that max-pool-fed layers pass their materialised pooled activation as RAW. */
int ebsdvae_conv3x3_wgrad_slices(int B, int H, int W, int cin, int cout);
int ebsdvae_conv3x3_wgrad(const float* src, const float* src_stats, int src_mode,
                          const float* gy, float* wpart, float* bpart, int B, int H, int W,
                          int cin, int cout, ebsdvae_stream_t stream);
/* work: device scratch of ebsdvae_wgrad_reduce_work(...) bytes (double partial sums) */
size_t ebsdvae_wgrad_reduce_work(int slices, int cin, int cout);
/* Split-bf16 weight gradient (pieces = 2 or 3, as ebsdvae_conv3x3_fwd_split): same partial
 * layout and reduction as ebsdvae_conv3x3_wgrad, 64-pixel tiles on
 * v_mfma_f32_16x16x32_bf16 with transposed LDS reads; cin % 32 == 0, cout 32 or 64k. */
int ebsdvae_conv3x3_wgrad_split_slices(int B, int H, int W, int cin, int cout, int pieces);
int ebsdvae_conv3x3_wgrad_split(const float* src, const float* src_stats, int src_mode,
                                const float* gy, float* wpart, float* bpart, int B, int H, int W,
                                int cin, int cout, int pieces, ebsdvae_stream_t stream);
/* Split-fp16 weight gradient (f16x3): as ebsdvae_conv3x3_wgrad_split with two fp16 pieces per
 * operand on v_mfma_f32_16x16x32_f16.  gy of each slice is scaled by 2^k (k from the maximum
 * of gmax over the images the slice covers, as ebsdvae_conv3x3_dgrad_inbwd_f16) and the
 * partials are unscaled; the bias partials sum the unscaled gy.  The activation operand is
 * not scaled, so src must be a normalised activation (NORM modes, or a materialised pooled
 * activation passed RAW).  Slices: ebsdvae_conv3x3_wgrad_split_slices(..., EBSDVAE_PIECES_F16). */
int ebsdvae_conv3x3_wgrad_f16(const float* src, const float* src_stats, int src_mode,
                              const float* gy, const float* gmax, int gm_tiles, float* wpart,
                              float* bpart, int B, int H, int W, int cin, int cout,
                              ebsdvae_stream_t stream);
/* Fused input + weight gradient of a 32 -> 32 layer whose source is the previous block's
 * normalised output (src_mode ACT_NORM: y_prev at H x W, its InstanceNorm-backward reduce routed
 * P_ID; ACT_NORM_UP: y_prev at H/2 x W/2, the input gradient 2x2-summed, P_UPSUM) in one pass
 * over gy and y_prev (encoder.1 / decoder.13 of latice/model.py:95-106): what
 * ebsdvae_conv3x3_dgrad_inbwd_f16(..., pmode) and ebsdvae_conv3x3_wgrad_f16 compute together.
 * wpack: the layer's split-fp16 input-gradient pack; gin (h = g * lrelu'(xhat_prev)) at
 * y_prev's resolution; part (B, T, 32) double2 with T = ebsdvae_conv3x3_dwgrad_stat_tiles(H, W)
 * (finalize over y_prev's H*W with ebsdvae_in_bwd_finalize); wpart / bpart
 * ebsdvae_conv3x3_dwgrad_slices(...) slice partials for ebsdvae_wgrad_reduce(_batch).
 * H == W, H / 8 a power of two. */
int ebsdvae_conv3x3_dwgrad_slices(int B, int H, int W, int cin, int cout);
int ebsdvae_conv3x3_dwgrad_stat_tiles(int H, int W);
int ebsdvae_conv3x3_dwgrad_f16(const float* gy, const float* gmax, int gm_tiles, const void* wpack,
                               const float* y_prev, const float* st_prev, int src_mode, float* gin,
                               double* part, float* wpart, float* bpart, int B, int H, int W,
                               int cin, int cout, ebsdvae_stream_t stream);
int ebsdvae_wgrad_reduce(const float* wpart, const float* bpart, int slices, float* dw,
                         float* db, int cin, int cout, int kind, void* work,
                         ebsdvae_stream_t stream);
/* Batched form: the slice reductions of n <= EBSDVAE_MAX_WGRAD_BATCH layers in two launches (the
 * per-layer form costs two launches per layer).  Each layer's result is bit-identical to
 * ebsdvae_wgrad_reduce.  descs live in HOST memory (passed to the kernels by value); work is
 * device scratch of ebsdvae_wgrad_reduce_batch_work(descs, n) bytes. */
#define EBSDVAE_MAX_WGRAD_BATCH 32
typedef struct {
  const float* wpart; /* device, [slices][tap][cout][cin] */
  const float* bpart; /* device, [slices][cout] */
  float* dw;          /* device, parameter layout of `kind` */
  float* db;          /* device or NULL */
  int slices, cin, cout, kind;
} ebsdvae_wgrad_reduce_desc;
size_t ebsdvae_wgrad_reduce_batch_work(const ebsdvae_wgrad_reduce_desc* descs, int n);
int ebsdvae_wgrad_reduce_batch(const ebsdvae_wgrad_reduce_desc* descs, int n, void* work,
                               ebsdvae_stream_t stream);

/* ---- InstanceNorm2d + LeakyReLU (latice/model.py:96-97,105-106) -----------------------
 * combine conv-epilogue partials {mean,M2} (tiles per image, n elements each) into
 * {mean, rstd} per (b,c). */
int ebsdvae_in_stats_finalize(const float* part, float* stats, int B, int C, int tiles,
                              int n_per_tile, ebsdvae_stream_t stream);
/* materialise act(src) at logical (B,H,W,C) NHWC (e.g. the encoder output after the last
 * MaxPool2d, latice/model.py:124) */
int ebsdvae_act_apply(const float* src, const float* src_stats, int src_mode, float* out,
                      int B, int H, int W, int C, ebsdvae_stream_t stream);
/* backward through [pool|upsample] . LeakyReLU . InstanceNorm of one block.
 * gnext: gradient w.r.t. the consumer's input; pmode 0 identity, 1 the consumer pooled
 * (gnext at H/2), 2 the consumer upsampled (gnext at 2H).  y/stats: the block's saved
 * pre-norm output and statistics.  Two passes: reduce -> bstats {mean(g_xhat),
 * mean(g_xhat*xhat)} per (b,c), then apply -> gy (conv-output gradient, (B,H,W,C)).
 * The plane sums are accumulated in double (part: B*tiles*C double2), as the reference's
 * CPU InstanceNorm backward does; the mean-subtraction cancels strongly. */
int ebsdvae_in_bwd_tiles(int H, int W, int C);
int ebsdvae_in_bwd_reduce(const float* gnext, int pmode, const float* y, const float* stats,
                          double* part, int B, int H, int W, int C, ebsdvae_stream_t stream);
int ebsdvae_in_bwd_finalize(const double* part, float* bstats, int B, int C, int tiles,
                            int HW, ebsdvae_stream_t stream);
int ebsdvae_in_bwd_apply(const float* gnext, int pmode, const float* y, const float* stats,
                         const float* bstats, float* gy, int B, int H, int W, int C,
                         ebsdvae_stream_t stream);
/* As ebsdvae_in_bwd_apply, and also writes gmax[b * T + t] = max |gy| over tile t of image b
 * (T = ebsdvae_in_bwd_apply_tiles(B, H, W, C) row bands per image; gmax may be NULL). */
int ebsdvae_in_bwd_apply_tiles(int B, int H, int W, int C);
int ebsdvae_in_bwd_apply_max(const float* gnext, int pmode, const float* y, const float* stats,
                             const float* bstats, float* gy, float* gmax, int B, int H, int W,
                             int C, ebsdvae_stream_t stream);
/* As ebsdvae_in_bwd_apply_max for h (a fused input gradient's output, routed like gnext):
 * the LeakyReLU factor is already in it.  gmax may be NULL. */
int ebsdvae_in_bwd_happly(const float* h, int pmode, const float* y, const float* stats,
                          const float* bstats, float* gy, float* gmax, int B, int H, int W, int C,
                          ebsdvae_stream_t stream);
/* Network-end fusions (C == 32; slices = B * ebsdvae_in_bwd_tiles(H,W,C) partials for
 * ebsdvae_wgrad_reduce):
 *  final_*: the block feeding the last conv (latice/model.py:147-148).  Its output gradient
 *    sum_tap g1[q-d(tap)] * w14[c][tap] is recomputed from the 1-channel logit gradient g1
 *    (never materialised); the reduce pass also emits that conv's dW (cin=32, cout=1) and
 *    db partials.
 *  first_apply_wgrad: the apply pass of the first block (latice/model.py:110) that
 *    accumulates the first conv's dW (cin=1, cout=32) and db partials against the input x
 *    instead of writing gy (x needs no gradient). */
int ebsdvae_in_bwd_final_reduce(const float* g1, const float* w14, const float* y,
                                const float* stats, double* part, float* wpart, float* bpart,
                                int B, int H, int W, int C, ebsdvae_stream_t stream);
int ebsdvae_in_bwd_final_apply(const float* g1, const float* w14, const float* y,
                               const float* stats, const float* bstats, float* gy, int B, int H,
                               int W, int C, ebsdvae_stream_t stream);
/* As ebsdvae_in_bwd_final_apply, and also writes gmax[b * T + t] = max |gy| over row band t
 * of image b, T = ebsdvae_in_bwd_final_tiles(H, W): the gradient scale of the split-fp16
 * input- and weight-gradient convs that consume gy. */
int ebsdvae_in_bwd_final_tiles(int H, int W);
int ebsdvae_in_bwd_final_apply_max(const float* g1, const float* w14, const float* y,
                                   const float* stats, const float* bstats, float* gy, float* gmax,
                                   int B, int H, int W, int C, ebsdvae_stream_t stream);
int ebsdvae_in_bwd_first_apply_wgrad(const float* gnext, const float* y, const float* stats,
                                     const float* bstats, const float* x, float* wpart,
                                     float* bpart, int B, int H, int W, int C,
                                     ebsdvae_stream_t stream);
/* As ebsdvae_in_bwd_first_apply_wgrad, with the first conv's output y0 recomputed from x, w0
 * (encoder.0 weight, (C,1,3,3)) and b0 (encoder.0 bias) instead of read: bit-identical to the
 * y0 that ebsdvae_conv_first_fwd wrote (one shared fma chain), 4*B*H*W*C bytes less traffic. */
int ebsdvae_in_bwd_first_apply_wgrad_rc(const float* gnext, const float* w0, const float* b0,
                                        const float* stats, const float* bstats, const float* x,
                                        float* wpart, float* bpart, int B, int H, int W, int C,
                                        ebsdvae_stream_t stream);
/* The first block's pass (the two above) on h, a fused input gradient's output */
int ebsdvae_in_bwd_first_happly_wgrad(const float* h, const float* y, const float* stats,
                                      const float* bstats, const float* x, float* wpart,
                                      float* bpart, int B, int H, int W, int C,
                                      ebsdvae_stream_t stream);
int ebsdvae_in_bwd_first_happly_wgrad_rc(const float* h, const float* w0, const float* b0,
                                         const float* stats, const float* bstats, const float* x,
                                         float* wpart, float* bpart, int B, int H, int W, int C,
                                         ebsdvae_stream_t stream);
/* gradient of nearest x2 upsampling: out[b,h,w,c] = sum of the 2x2 block of g (at 2H) */
int ebsdvae_upsample2_bwd(const float* g, float* out, int B, int H, int W, int C,
                          ebsdvae_stream_t stream);

/* ---- latent heads + reparameterisation (latice/model.py:55-64, 25-38) ----------------
 * enc: encoder output (B,S,S,C) NHWC.  flat = enc in NCHW flatten order (saved for
 * backward); mu/logvar = Linear(F,L); std = exp(logvar/2); z = mu + eps*std;
 * dec_in = Linear(L,F)(z) viewed (B,C,S,S) and written NHWC. */
/* work: ebsdvae_heads_work(B,C,S,L) bytes of caller-owned device scratch (split-K partial
 * sums over the S*S feature pixels; shared by heads_fwd / latent_mu / heads_bwd on one
 * stream).  C: a power of two in 16..256; L <= 64. */
size_t ebsdvae_heads_work(int B, int C, int S, int L);
int ebsdvae_heads_fwd(const float* enc, const float* w_mu, const float* b_mu,
                      const float* w_lv, const float* b_lv, const float* w_l2,
                      const float* b_l2, const float* eps, float* flat, float* mu,
                      float* std, float* z, float* dec_in, void* work, int B, int C, int S,
                      int L, ebsdvae_stream_t stream);
/* Encoder-only inference head: mu = Linear(F,L)(flatten_NCHW(enc)) (latice/model.py:55-58;
 * DiffractionPatternIndexer.build_dictionary consumes mu alone). */
int ebsdvae_latent_mu(const float* enc, const float* w_mu, const float* b_mu, float* mu,
                      void* work, int B, int C, int S, int L, ebsdvae_stream_t stream);
/* g_dec: grad of dec_in (B,S,S,C NHWC); g_z/g_mu/g_std: direct output grads (may be
 * NULL = 0).  Writes g_enc (B,S,S,C NHWC) and per-sample scratch
 * gs = [g_mu_tot (B,L) | g_logvar (B,L) | g_out (B,F)] consumed by heads_wgrad. */
int ebsdvae_heads_bwd(const float* g_dec, const float* g_z, const float* g_mu,
                      const float* g_std, const float* std, const float* eps,
                      const float* w_mu, const float* w_lv, const float* w_l2, float* g_enc,
                      float* gs, void* work, int B, int C, int S, int L,
                      ebsdvae_stream_t stream);
/* Weight/bias gradients of the three Linear heads (autograd's addmm backward for
 * latice/model.py:127-131): deterministic split-batch reduction through `work`
 * (ebsdvae_heads_wgrad_work(B,F,L) bytes, caller-owned). */
size_t ebsdvae_heads_wgrad_work(int B, int F, int L);
int ebsdvae_heads_wgrad(const float* flat, const float* z, const float* gs, float* gw_mu,
                        float* gb_mu, float* gw_lv, float* gb_lv, float* gw_l2,
                        float* gb_l2, void* work, int B, int F, int L,
                        ebsdvae_stream_t stream);

/* generic Linear (y = x W^T + b), for direct calls of model.mu / .logvar / .linear2 */
int ebsdvae_linear_fwd(const float* x, const float* w, const float* b, float* y, int M,
                       int K, int N, ebsdvae_stream_t stream);
int ebsdvae_linear_bwd(const float* x, const float* w, const float* gy, float* gx,
                       float* gw, float* gb, int M, int K, int N, ebsdvae_stream_t stream);
/* VariationalAutoEncoder.reparameterize (latice/model.py:25-38) */
int ebsdvae_reparam_fwd(const float* mu, const float* logvar, const float* eps, float* z,
                        float* std, int64_t n, ebsdvae_stream_t stream);
int ebsdvae_reparam_bwd(const float* gz, const float* gstd, const float* eps,
                        const float* std, float* gmu, float* glogvar, int64_t n,
                        ebsdvae_stream_t stream);
/* standard-normal sampler (counter-based Philox4x32-10 + Box-Muller) for eps
 * (replaces torch.distributions.Normal.rsample's normal_, latice/model.py:36-37).
 * If counter != NULL (device uint64), it is incremented first and the draw uses
 * offset + counter * ceil(n/4) as its Philox counter base, so a captured graph draws
 * fresh noise on every replay. */
int ebsdvae_normal_fill(float* out, int64_t n, uint64_t seed, uint64_t offset,
                        uint64_t* counter, ebsdvae_stream_t stream);

/* ---- loss (latice/lightning_module.py:79-156) ----------------------------------------
 * recon_b = mean_p BCEWithLogits(x_hat, x); kl_b = kl_lambda * mean_j [0.5 z^2 -
 * 0.5 ((z-mu)/std)^2 - log std]; elbo_b = kl_b + recon_b;
 * loss = mean elbo, kl_loss = mean kl, recon_loss = mean recon (device scalars). */
int ebsdvae_vae_loss_fwd(const float* x_hat, const float* x, const float* z, const float* mu,
                         const float* std, float kl_lambda, float* elbo, float* kl,
                         float* recon, float* loss, float* kl_loss, float* recon_loss, int B,
                         int P, int L, ebsdvae_stream_t stream);
/* upstream gradients g_loss, g_kl_loss, g_recon_loss (device scalars) and g_elbo (B) may
 * each be NULL (= 0); scale multiplies all of them (e.g. 1/world_size for data
 * parallelism).  g_x (gradient w.r.t. the BCE target) may be NULL.  g_xhat may be NULL (then
 * x_hat and x may be too): only the KL gradients g_z, g_mu, g_std are written (the training
 * step's logit gradient comes from ebsdvae_net_end). */
int ebsdvae_vae_loss_bwd(const float* x_hat, const float* x, const float* z, const float* mu,
                         const float* std, float kl_lambda, const float* g_loss,
                         const float* g_kl_loss, const float* g_recon_loss,
                         const float* g_elbo, float scale, float* g_xhat, float* g_z,
                         float* g_mu, float* g_std, float* g_x, int B, int P, int L,
                         ebsdvae_stream_t stream);

/* As ebsdvae_vae_loss_fwd with recon_b = sum_t bce_part[b][t] / P from the per-row-band BCE
 * sums of ebsdvae_net_end (tiles = ebsdvae_net_end_tiles(H, W)). */
int ebsdvae_vae_loss_fwd_parts(const float* bce_part, int tiles, const float* z, const float* mu,
                               const float* std, float kl_lambda, float* elbo, float* kl,
                               float* recon, float* loss, float* kl_loss, float* recon_loss, int B,
                               int P, int L, ebsdvae_stream_t stream);

/* ---- network end of the training step (latice/model.py:147-148 + lightning_module.py:79-92) --
 * One pass over the last block's pre-norm output y13 (B, H, W, C) NHWC with its statistics
 * st13 {mean, rstd} (B, C), for C == 32, W == 128 or 256, H % 32 == 0 (row bands of 64 rows
 * where H % 64 == 0, else 32; T = ebsdvae_net_end_tiles(H, W)):
 *   x_hat (B, 1, H, W) = Conv2d(32, 1)(lrelu(IN(y13))) with w14 (1, 32, 3, 3), b14 (1) or NULL;
 *   g1 (B, H, W) = g_loss * scale / (B * H * W) * (sigmoid(x_hat) - x), the gradient of the
 *     mean-BCE part of the loss w.r.t. the logits (g_loss a device scalar, NULL = 1);
 *   bce_part (B, T): per row band the sum of BCE-with-logits(x_hat, x);
 *   part (B, T, C) double2: the InstanceNorm-backward reduce sums of the last block with its
 *     output gradient recomputed from g1 (as ebsdvae_in_bwd_final_reduce; finalize with
 *     ebsdvae_in_bwd_finalize(part, ..., T, H * W));
 *   wpart (B * T, 9, 1, C) / bpart (B * T): the final conv's weight / bias gradient slices for
 *     ebsdvae_wgrad_reduce (cin C, cout 1, kind 0).
 * T = ebsdvae_net_end_tiles(H, W) (-1: shape unsupported).  Replaces ebsdvae_conv3x3_cout1_fwd,
 * the BCE part of ebsdvae_vae_loss_fwd / _bwd and ebsdvae_in_bwd_final_reduce, which read y13
 * once each.  The three contractions run on the split-fp16 MFMA (f16x3 products); the reduce
 * sums come from the weight-gradient contraction and an indicator contraction
 * (s2 = sum_t w G, s1 = sum_t w (slope S + (1 - slope) P), net_end.hip).
 * ebsdvae_net_end_valu: the same outputs from the fp32 VALU form (round 5; A/B). */
int ebsdvae_net_end_tiles(int H, int W);
int ebsdvae_net_end(const float* y13, const float* st13, const float* w14, const float* b14,
                    const float* x, const float* g_loss, float scale, float* x_hat, float* g1,
                    float* bce_part, double* part, float* wpart, float* bpart, int B, int H, int W,
                    int C, ebsdvae_stream_t stream);
int ebsdvae_net_end_valu(const float* y13, const float* st13, const float* w14, const float* b14,
                    const float* x, const float* g_loss, float scale, float* x_hat, float* g1,
                    float* bce_part, double* part, float* wpart, float* bpart, int B, int H, int W,
                    int C, ebsdvae_stream_t stream);

/* ---- optimiser (torch.optim.Adam semantics; latice/lightning_module.py:26-28) ---------
 * state: device float step counter (incremented by this call), m, v, vmax (amsgrad). */
int ebsdvae_adam(float* p, const float* g, float* m, float* v, float* vmax, float* step,
                 int64_t n, float lr, float beta1, float beta2, float eps,
                 float weight_decay, int amsgrad, ebsdvae_stream_t stream);

/* ---- latent dictionary search ---------------------------
 * GPU form of latice/index/faiss_db.py's IndexFlatIP cosine search: rows are L2-normalised
 * (norm 0 -> 1, faiss_db.py:107-111) and queried exhaustively by inner product.
 * ebsdvae_cosine_topk writes, per query q, the k (1..64, <= N) best dictionary rows ordered
 * by (score desc, row index asc): out_scores[q][k] (fp32), out_idx[q][k] (int64).  d is 16,
 * 32 or 64; db is N x d row-major, queries Q x d, both already normalised.  work: device
 * scratch of ebsdvae_cosine_topk_work(N, Q, d, k) bytes. */
int ebsdvae_l2_normalize_rows(const float* x, float* y, long long n, int d,
                              ebsdvae_stream_t stream);
size_t ebsdvae_cosine_topk_work(long long N, int Q, int d, int k);
int ebsdvae_cosine_topk(const float* db, long long N, const float* queries, int Q, int d, int k,
                        float* out_scores, long long* out_idx, void* work,
                        ebsdvae_stream_t stream);

/* ---- orientation consensus ------------------------------
 * Batched latice/index/faiss_db.py:258-398 find_best_orientation (== chroma_db.py:261-375):
 * query q's candidates are orientations[cand_idx[q][0..n-1]] (ZXZ Euler degrees, float64,
 * top-n match order; n <= 64).  Writes best[q][3] (the symmetry-resolved mean on success,
 * else candidate 0), mean[q][3] (NaN when no consensus), success[q] (0/1) and
 * similar_mask[q] (bit j = candidate j within threshold_deg of the last reference tried). */
int ebsdvae_orient_consensus(const double* orientations, const long long* cand_idx, int Q, int n,
                             double threshold_deg, int min_matches, int max_iterations,
                             double* best, double* mean, int* success,
                             unsigned long long* similar_mask, ebsdvae_stream_t stream);

/* ---- pattern ingest -------------------------------------
 * Batched DPdataset.__getitem__ transform (latice/data_module.py:17-33,125-133): raw
 * (B, H0, W0) patterns (src_dtype 0 = float64, 1 = float32) -> uint8(x * 255) -> centre
 * crop / zero-pad to (out_h, out_w) as torchvision's CenterCrop -> float32 / 255, written as
 * dst (B, 1, out_h, out_w).  Values outside [0, 1] are clamped before the uint8 cast. */
int ebsdvae_ingest_patterns(const void* src, int src_dtype, int B, int H0, int W0, int out_h,
                            int out_w, float* dst, ebsdvae_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* EBSDVAE_H_ */
