// Host-side AddressSanitizer driver for libebsdvae's C ABI (the library's
// argument validation, scratch-size queries and error plumbing run on the host before any
// launch).  Linked with the library objects built with -Xarch_host -fsanitize=address
// (ebsd-vae_amd/build.py --asan); needs no GPU: every call below is a shape / size query or is
// rejected by validation.  Exit 0 = all expectations held (ASan aborts on any memory error).
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/ebsdvae.h"

static int g_fail = 0;

static void expect_err(int rc, const char* what) {
  const char* e = ebsdvae_last_error();
  if (rc == 0 || e == nullptr || strlen(e) == 0 || strlen(e) >= 512) {
    printf("FAIL %s: rc=%d err='%s'\n", what, rc, e ? e : "(null)");
    ++g_fail;
  }
}

int main() {
  if (ebsdvae_version() != EBSDVAE_ABI_VERSION) { printf("FAIL version\n"); return 1; }
  const int sizes[] = {-8, 0, 1, 4, 7, 8, 16, 32, 64, 100, 128, 256, 512, 4096, 1 << 20};
  const int chans[] = {-1, 0, 1, 3, 8, 16, 32, 64, 96, 128, 256};
  const int pieces[] = {-1, 0, 1, 2, 3, EBSDVAE_PIECES_F16, 99};
  long long acc = 0;
  for (int H : sizes) {
    acc += ebsdvae_conv_first_stat_tiles(H, H) + ebsdvae_in_bwd_final_tiles(H, H);
    for (int C : chans) {
      acc += ebsdvae_conv3x3_stat_tiles(H, H, C) + ebsdvae_conv3x3_split_stat_tiles(H, H, C) +
             ebsdvae_in_bwd_tiles(H, H, C);
      for (int B : {0, 1, 3, 256, 1024})
        acc += ebsdvae_in_bwd_apply_tiles(B, H, H, C);
      for (int C2 : chans) {
        for (int B : {0, 1, 2, 256, 1024})
          acc += ebsdvae_conv3x3_wgrad_slices(B, H, H, C, C2);
        for (int p : pieces) {
          acc += ebsdvae_conv3x3_split_supported(H, H, C, C2, p) +
                 ebsdvae_conv3x3_split_pool_ok(H, H, C, C2, p);
          for (int B : {1, 256})
            acc += ebsdvae_conv3x3_wgrad_split_slices(B, H, H, C, C2, p);
        }
      }
    }
  }
  for (int C : chans)
    for (int C2 : chans)
      for (int p : pieces) acc += (long long)(ebsdvae_pack_split_bytes(C, C2, p) & 0xffff);
  for (int s : {-1, 0, 1, 64, 4096})
    for (int C : chans) acc += (long long)(ebsdvae_wgrad_reduce_work(s, C, 32) & 0xffff);
  for (int B : {-1, 0, 1, 256})
    for (int F : {0, 2048, 8192}) acc += (long long)(ebsdvae_heads_wgrad_work(B, F, 16) & 0xffff);
  for (long long N : {0LL, 1LL, 1000LL, 1LL << 20})
    for (int k : {0, 1, 20, 64, 65}) acc += (long long)(ebsdvae_cosine_topk_work(N, 4096, 16, k) & 0xffff);

  // batched descriptors: sizes from host arrays, including n at and past the limits
  std::vector<ebsdvae_wgrad_reduce_desc> wd(EBSDVAE_MAX_WGRAD_BATCH + 1);
  for (size_t i = 0; i < wd.size(); ++i) {
    wd[i] = {};
    wd[i].slices = (int)(i * 7 % 300);
    wd[i].cin = 32;
    wd[i].cout = 64;
  }
  acc += (long long)(ebsdvae_wgrad_reduce_batch_work(wd.data(), EBSDVAE_MAX_WGRAD_BATCH) & 0xffff);
  expect_err(ebsdvae_wgrad_reduce_batch(wd.data(), EBSDVAE_MAX_WGRAD_BATCH + 1, nullptr, nullptr),
             "wgrad_reduce_batch n > max");
  expect_err(ebsdvae_wgrad_reduce_batch(nullptr, 3, nullptr, nullptr), "wgrad_reduce_batch null");
  std::vector<ebsdvae_pack_desc> pd(EBSDVAE_MAX_PACK + 1);
  for (auto& d : pd) d = {nullptr, nullptr, 32, 32, 0, 0};
  expect_err(ebsdvae_pack_conv_weights(pd.data(), EBSDVAE_MAX_PACK + 1, nullptr), "pack n > max");
  expect_err(ebsdvae_pack_conv_weights_split(pd.data(), EBSDVAE_MAX_PACK + 1, 2, nullptr),
             "pack_split n > max");
  expect_err(ebsdvae_pack_conv_weights_split(pd.data(), 2, 2, nullptr), "pack_split null ptrs");

  // argument validation: null pointers and unsupported shapes, rejected before any launch
  expect_err(ebsdvae_conv3x3_fwd(nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr,
                                 2, 16, 16, 3, 32, nullptr), "conv3x3_fwd cin=3");
  expect_err(ebsdvae_conv3x3_fwd_split(nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                                       nullptr, 2, 128, 128, 32, 32, 99, nullptr), "fwd_split pieces");
  expect_err(ebsdvae_conv3x3_fwd_split_st(nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                                          nullptr, nullptr, 2, 128, 128, 32, 32,
                                          EBSDVAE_PIECES_F16, nullptr), "fwd_split_st null");
  expect_err(ebsdvae_conv3x3_dgrad_inbwd_f16_bst(nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                                                 nullptr, 0, nullptr, nullptr, 0, 2, 128, 128, 32,
                                                 32, nullptr), "dgrad_f16_bst null");
  expect_err(ebsdvae_conv3x3_wgrad_f16(nullptr, nullptr, 1, nullptr, nullptr, 0, nullptr, nullptr,
                                       2, 128, 128, 32, 32, nullptr), "wgrad_f16 null");
  expect_err(ebsdvae_conv3x3_wgrad(nullptr, nullptr, 0, nullptr, nullptr, nullptr, 2, 5, 5, 32, 32,
                                   nullptr), "wgrad odd shape");
  expect_err(ebsdvae_conv_first_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, 2, 128, 128, 32,
                                    nullptr), "conv_first null");
  expect_err(ebsdvae_conv3x3_cout1_fwd(nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, 2, 128,
                                       128, 32, nullptr), "cout1 null");
  expect_err(ebsdvae_heads_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                               nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 2, 128,
                               4, 16, nullptr), "heads_fwd null");
  if (ebsdvae_heads_work(256, 128, 4, 16) != (size_t)16 * 256 * 32 * 4 ||
      ebsdvae_heads_work(2, 96, 4, 16) != 0 || ebsdvae_heads_work(2, 128, 4, 65) != 0) {
    printf("FAIL heads_work\n");
    ++g_fail;
  }
  expect_err(ebsdvae_in_bwd_reduce(nullptr, 0, nullptr, nullptr, nullptr, 2, 128, 128, 32, nullptr),
             "in_bwd_reduce null");
  expect_err(ebsdvae_in_bwd_apply_max(nullptr, 9, nullptr, nullptr, nullptr, nullptr, nullptr, 2,
                                      128, 128, 32, nullptr), "in_bwd_apply_max pmode");
  expect_err(ebsdvae_vae_loss_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, nullptr,
                                  nullptr, nullptr, nullptr, nullptr, nullptr, 2, 16384, 16,
                                  nullptr), "loss_fwd null");
  expect_err(ebsdvae_adam(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 100, 1e-4f, 0.9f,
                          0.999f, 1e-8f, 0.f, 0, nullptr), "adam null");
  expect_err(ebsdvae_cosine_topk(nullptr, 10, nullptr, 1, 16, 65, nullptr, nullptr, nullptr,
                                 nullptr), "topk k=65");
  expect_err(ebsdvae_orient_consensus(nullptr, nullptr, 1, 65, 3.0, 3, 5, nullptr, nullptr, nullptr,
                                      nullptr, nullptr), "orient n=65");
  expect_err(ebsdvae_ingest_patterns(nullptr, 7, 2, 140, 140, 128, 128, nullptr, nullptr),
             "ingest dtype");
  expect_err(ebsdvae_normal_fill(nullptr, 16, 1, 0, nullptr, nullptr), "normal null");
  for (int H : sizes) acc += ebsdvae_net_end_tiles(H, 128) + ebsdvae_net_end_tiles(H, H);
  expect_err(ebsdvae_net_end(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1.f, nullptr,
                             nullptr, nullptr, nullptr, nullptr, nullptr, 2, 128, 128, 32, nullptr),
             "net_end null");
  expect_err(ebsdvae_vae_loss_fwd_parts(nullptr, 8, nullptr, nullptr, nullptr, 0.f, nullptr, nullptr,
                                        nullptr, nullptr, nullptr, nullptr, 2, 16384, 16, nullptr),
             "loss_fwd_parts null");
  printf("abi_asan: %s (query checksum %lld)\n", g_fail ? "FAILED" : "ok", acc);
  return g_fail ? 1 : 0;
}
