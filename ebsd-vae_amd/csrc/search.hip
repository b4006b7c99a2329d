// Exact cosine top-k over a latent dictionary: the GPU form of
// the reference's FAISS IndexFlatIP search on L2-normalised vectors
// (latice/index/faiss_db.py:107-111 _l2_normalize, :160-174 add_vectors, :216-256
// query_similar; faiss-cpu 1.10 IndexFlatIP = exhaustive inner product, k best by score).
//
//   ebsdvae_l2_normalize_rows   v / ||v||_2 per row (zero rows stay zero: norm 0 -> 1)
//   ebsdvae_cosine_topk         per query: the k dictionary rows of largest <q, db_i>,
//                               ordered by (score desc, index asc)
//
// HBM-bound: one pass over the dictionary (N x D fp32, D <= 64) per group of queries.  A wave
// owns QW queries and one chunk of dictionary rows; each lane scores one row per 64-row
// step (the row is one contiguous D*4-byte record, so a wave reads 64 consecutive rows), and
// the wave keeps each query's running top-k in registers -- slot s in lane s -- with its
// current minimum as an admission threshold: a row is inserted only if it beats that
// threshold (ballot), so after the first few thousand rows almost nothing is inserted.
// Chunks' lists are merged per query by the same insertion in a second launch, then
// bitonic-sorted across the wave.  Ties break to the lower row index (deterministic).
#include "common.h"
#include "../../include/ebsdvae.h"

#include <float.h>

namespace ev {

constexpr int TK_WAVES = 4;     // waves per block (each its own query group, same chunk)
constexpr int TK_MAXK = 64;
constexpr int TK_MAXD = 64;

// (s, i) beats (t, j)
EV_DEVINL bool tk_better(float s, int i, float t, int j) { return s > t || (s == t && i < j); }

// running top-k of one query in one wave: lane l < k holds slot l
struct TopK {
  float v;
  int i;
  float thr;   // wave-uniform: the worst kept slot (admission threshold)
  int thr_i;
  int thr_lane;
};

EV_DEVINL void tk_init(TopK& t, int k, int lane) {
  t.v = -FLT_MAX;
  t.i = 0x7fffffff;
  (void)k;
  (void)lane;
  t.thr = -FLT_MAX;
  t.thr_i = 0x7fffffff;
  t.thr_lane = 0;
}

// recompute the worst slot among lanes < k (wave reduction, ties -> larger index is worse)
EV_DEVINL void tk_refresh(TopK& t, int k, int lane) {
  float v = lane < k ? t.v : FLT_MAX;
  int i = lane < k ? t.i : -1;
  int l = lane;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    const int l2 = __shfl_xor(l, o, 64);
    // keep the WORSE of the two (the one the other beats)
    if (tk_better(v, i, v2, i2) || (v == v2 && i == i2 && l2 < l)) { v = v2; i = i2; l = l2; }
  }
  t.thr = v;
  t.thr_i = i;
  t.thr_lane = l;
}

// offer candidate (s, idx) held by each lane (valid where ok); inserts the qualifying ones
EV_DEVINL void tk_offer(TopK& t, float s, int idx, bool ok, int k, int lane) {
  unsigned long long m = __ballot(ok && tk_better(s, idx, t.thr, t.thr_i));
  while (m) {
    const int src = __builtin_ctzll(m);
    m &= m - 1;
    const float cs = __shfl(s, src, 64);
    const int ci = __shfl(idx, src, 64);
    if (!tk_better(cs, ci, t.thr, t.thr_i)) continue;   // threshold rose meanwhile
    if (lane == t.thr_lane) { t.v = cs; t.i = ci; }
    tk_refresh(t, k, lane);
  }
}

// bitonic sort of the 64 lanes' (v, i), best first (slots >= k hold -FLT_MAX / INT_MAX)
EV_DEVINL void tk_sort(float& v, int& i, int lane) {
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float v2 = __shfl_xor(v, stride, 64);
      const int i2 = __shfl_xor(i, stride, 64);
      const bool asc = (lane & size) == 0;          // this block orders best-first
      const bool lower = (lane & stride) == 0;
      const bool take = (lower == asc) ? tk_better(v2, i2, v, i) : tk_better(v, i, v2, i2);
      if (take) { v = v2; i = i2; }
    }
  }
}

__global__ __launch_bounds__(256) void l2norm_rows_kernel(const float* __restrict__ x,
                                                          float* __restrict__ y, long long n, int d) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* p = x + r * d;
  float s = 0.f;
  for (int j = 0; j < d; ++j) s = fmaf(p[j], p[j], s);
  float nr = sqrtf(s);
  if (nr == 0.f) nr = 1.f;
  for (int j = 0; j < d; ++j) y[r * d + j] = p[j] / nr;
}

// queries per wave: their D-float vectors live in VGPRs (64 per wave at any D)
template <int D>
constexpr int tk_qw() { return 64 / D; }

// pass 1: grid (chunks, ceil(Q / (QW * TK_WAVES))); partial lists [q][chunk][k]
template <int D>
__global__ __launch_bounds__(256) void topk_chunk_kernel(const float* __restrict__ db, long long N,
                                                         const float* __restrict__ qv, int Q, int k,
                                                         long long rows_per_chunk, int nchunk,
                                                         float* __restrict__ ps, int* __restrict__ pi) {
  constexpr int TK_QW = tk_qw<D>();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q0 = (blockIdx.y * TK_WAVES + wave) * TK_QW;
  if (q0 >= Q) return;
  const int chunk = blockIdx.x;
  const long long r0 = (long long)chunk * rows_per_chunk;
  const long long r1 = r0 + rows_per_chunk < N ? r0 + rows_per_chunk : N;
  float qr[TK_QW][D];
#pragma unroll
  for (int a = 0; a < TK_QW; ++a)
#pragma unroll
    for (int j = 0; j < D; ++j) qr[a][j] = (q0 + a < Q) ? qv[(size_t)(q0 + a) * D + j] : 0.f;
  TopK t[TK_QW];
#pragma unroll
  for (int a = 0; a < TK_QW; ++a) tk_init(t[a], k, lane);
  for (long long rb = r0; rb < r1; rb += 64) {
    const long long r = rb + lane;
    const bool ok = r < r1;
    float rowv[D];
    const float4* rp = reinterpret_cast<const float4*>(db + (ok ? r : r0) * D);
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
      const float4 v = rp[j];
      rowv[4 * j] = v.x; rowv[4 * j + 1] = v.y; rowv[4 * j + 2] = v.z; rowv[4 * j + 3] = v.w;
    }
#pragma unroll
    for (int a = 0; a < TK_QW; ++a) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < D; ++j) s = fmaf(qr[a][j], rowv[j], s);
      tk_offer(t[a], s, (int)r, ok && (q0 + a < Q), k, lane);
    }
  }
#pragma unroll
  for (int a = 0; a < TK_QW; ++a) {
    if (q0 + a >= Q || lane >= k) continue;
    const size_t o = ((size_t)(q0 + a) * nchunk + chunk) * k + lane;
    ps[o] = t[a].v;
    pi[o] = t[a].i;
  }
}

// pass 2: one wave per query merges nchunk partial lists, sorts, writes k results
__global__ __launch_bounds__(64) void topk_merge_kernel(const float* __restrict__ ps,
                                                        const int* __restrict__ pi, int nchunk, int k,
                                                        float* __restrict__ out_s,
                                                        long long* __restrict__ out_i) {
  const int q = blockIdx.x, lane = threadIdx.x;
  TopK t;
  tk_init(t, k, lane);
  const size_t base = (size_t)q * nchunk * k;
  const int total = nchunk * k;
  for (int c0 = 0; c0 < total; c0 += 64) {
    const int c = c0 + lane;
    const bool ok = c < total;
    const float s = ok ? ps[base + c] : -FLT_MAX;
    const int i = ok ? pi[base + c] : 0x7fffffff;
    tk_offer(t, s, i, ok && i != 0x7fffffff, k, lane);
  }
  float v = lane < k ? t.v : -FLT_MAX;
  int i = lane < k ? t.i : 0x7fffffff;
  tk_sort(v, i, lane);
  if (lane < k) {
    out_s[(size_t)q * k + lane] = v;
    out_i[(size_t)q * k + lane] = (i == 0x7fffffff) ? -1 : (long long)i;
  }
}

static int topk_chunks(long long N, int Q, int d) {
  // enough (chunk, query-group) waves to fill the chip, chunks of >= 512 rows
  const int qw = 64 / d;
  const int qg = (Q + qw * TK_WAVES - 1) / (qw * TK_WAVES);
  long long c = (2048 + qg - 1) / qg;
  const long long cmax = (N + 511) / 512;
  if (c > cmax) c = cmax;
  if (c < 1) c = 1;
  if (c > 4096) c = 4096;
  return (int)c;
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_l2_normalize_rows(const float* x, float* y, long long n, int d,
                                         ebsdvae_stream_t stream) {
  EV_REQUIRE(x && y && n >= 0 && d > 0, "l2_normalize_rows: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, x, y, n, d);
  return evh::check_launch("l2_normalize_rows");
}

extern "C" size_t ebsdvae_cosine_topk_work(long long N, int Q, int d, int k) {
  if (N <= 0 || Q <= 0 || k <= 0 || !(d == 16 || d == 32 || d == 64)) return 0;
  const int nc = topk_chunks(N, Q, d);
  return (size_t)Q * nc * k * (sizeof(float) + sizeof(int));
}

extern "C" int ebsdvae_cosine_topk(const float* db, long long N, const float* queries, int Q, int d,
                                   int k, float* out_scores, long long* out_idx, void* work,
                                   ebsdvae_stream_t stream) {
  EV_REQUIRE(db && queries && out_scores && out_idx && work, "cosine_topk: null pointer");
  EV_REQUIRE(N > 0 && N < 0x7fffffffLL && Q > 0, "cosine_topk: N=%lld Q=%d out of range", N, Q);
  EV_REQUIRE(k >= 1 && k <= TK_MAXK && k <= N, "cosine_topk: k=%d (1..%d, <= N)", k, TK_MAXK);
  EV_REQUIRE(d == 16 || d == 32 || d == 64, "cosine_topk: d=%d (16, 32 or 64)", d);
  const int nc = topk_chunks(N, Q, d);
  const long long rpc = (N + nc - 1) / nc;
  float* ps = reinterpret_cast<float*>(work);
  int* pi = reinterpret_cast<int*>(ps + (size_t)Q * nc * k);
  const int qw = 64 / d;
  const dim3 grid(nc, (Q + qw * TK_WAVES - 1) / (qw * TK_WAVES));
  hipStream_t s = (hipStream_t)stream;
  if (d == 16)
    hipLaunchKernelGGL(topk_chunk_kernel<16>, grid, dim3(256), 0, s, db, N, queries, Q, k, rpc, nc, ps, pi);
  else if (d == 32)
    hipLaunchKernelGGL(topk_chunk_kernel<32>, grid, dim3(256), 0, s, db, N, queries, Q, k, rpc, nc, ps, pi);
  else
    hipLaunchKernelGGL(topk_chunk_kernel<64>, grid, dim3(256), 0, s, db, N, queries, Q, k, rpc, nc, ps, pi);
  hipLaunchKernelGGL(topk_merge_kernel, dim3(Q), dim3(64), 0, s, ps, pi, nc, k, out_scores, out_idx);
  return evh::check_launch("cosine_topk");
}
