// Which CUs does a CU-masked stream (hipExtStreamCreateWithCUMask) run on, on MI355X?
// Launches 4096 one-wave blocks on a stream masked to the first N bits of the mask, each
// recording its XCC id and hardware CU id (s_getreg HW_REG_HW_ID / XCC_ID); prints how many
// distinct (XCC, SE, CU) slots and XCCs were used, per mask.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID (gfx9: id 4)
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    // keep the CU busy a little so blocks spread
    for (volatile int i = 0; i < 2000; ++i) {}
  }
}

static void run(const std::vector<uint32_t>& mask, const char* label) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    printf("%s: hipExtStreamCreateWithCUMask failed\n", label);
    return;
  }
  const int nb = 4096;
  unsigned* d;
  (void)hipMalloc(&d, nb * 8);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d);
  (void)hipStreamSynchronize(s);
  std::vector<unsigned> h(2 * nb);
  (void)hipMemcpy(h.data(), d, nb * 8, hipMemcpyDeviceToHost);
  std::set<unsigned> cus, xccs;
  std::vector<int> per_xcc(16, 0);
  for (int i = 0; i < nb; ++i) {
    const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xf;
    // gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    const unsigned key = (xcc << 16) | (se << 8) | (sh << 4) | cu;
    if (!cus.count(key)) per_xcc[xcc]++;
    cus.insert(key);
    xccs.insert(xcc);
  }
  printf("%s: %zu distinct CUs, %zu XCCs; CUs per XCC:", label, cus.size(), xccs.size());
  for (int x = 0; x < 8; ++x) printf(" %d", per_xcc[x]);
  printf("\n");
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs: %d\n", ncu);
  const int words = (ncu + 31) / 32;
  for (int n : {256, 192, 128, 64, 32, 8}) {
    std::vector<uint32_t> m(words, 0);
    for (int i = 0; i < n && i < ncu; ++i) m[i / 32] |= 1u << (i % 32);
    char lab[64];
    snprintf(lab, sizeof lab, "first %d bits", n);
    run(m, lab);
  }
  {  // every 4th bit
    std::vector<uint32_t> m(words, 0);
    for (int i = 0; i < ncu; i += 4) m[i / 32] |= 1u << (i % 32);
    run(m, "every 4th bit (64)");
  }
  {  // complement of first 192
    std::vector<uint32_t> m(words, 0);
    for (int i = 192; i < ncu; ++i) m[i / 32] |= 1u << (i % 32);
    run(m, "bits 192..255 (64)");
  }
  return 0;
}
