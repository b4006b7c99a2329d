// Streaming-store width micro-benchmark: 536 MB (B=256 x 128x128 x 32 ch fp32) written as
//  (a) the MFMA epilogue pattern: 4-byte stores, lane = channel, 2 pixels (2 x 128 B) per
//      wave instruction;
//  (b) 16-byte stores, 8 lanes per 128-B pixel, 8 pixels (1 KB) per wave instruction.
// hipcc --offload-arch=gfx950 -O3 tools/micro/store_width.hip -o /tmp/store_width
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void st4(float* __restrict__ y, size_t npix) {
  const int lane = threadIdx.x & 63, l32 = lane & 31, hk = lane >> 5;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = (gridDim.x * (size_t)blockDim.x) >> 6;
  for (size_t p0 = wave * 32; p0 < npix; p0 += nw * 32)   // 32 pixels per wave per round
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const size_t p = p0 + (r & 3) + 8 * (r >> 2) + 4 * hk;
      y[p * 32 + l32] = (float)r;
    }
}

__global__ void st16(float* __restrict__ y, size_t npix) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = (gridDim.x * (size_t)blockDim.x) >> 6;
  for (size_t p0 = wave * 32; p0 < npix; p0 += nw * 32)
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // 4 x 8 pixels
      const size_t p = p0 + 8 * i + (lane >> 3);
      reinterpret_cast<float4*>(y + p * 32)[lane & 7] = make_float4(i, 1.f, 2.f, 3.f);
    }
}

int main() {
  const size_t npix = (size_t)256 * 128 * 128;
  float* y;
  if (hipMalloc(&y, npix * 32 * 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int blocks : {1024, 4096, 16384}) {
    for (int k = 0; k < 2; ++k) {
      float best = 1e9;
      for (int rep = 0; rep < 20; ++rep) {
        hipEventRecord(a);
        if (k == 0) hipLaunchKernelGGL(st4, dim3(blocks), dim3(256), 0, 0, y, npix);
        else hipLaunchKernelGGL(st16, dim3(blocks), dim3(256), 0, 0, y, npix);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("%s blocks %6d: %8.1f us  %.2f TB/s\n", k ? "16B" : " 4B", blocks, best * 1e3,
             npix * 128.0 / (best * 1e-3) / 1e12);
    }
  }
  hipFree(y);
  return 0;
}
