// On-device pattern ingest: the reference's per-sample CPU
// transform of DPdataset.__getitem__ (latice/data_module.py:125-133 + the default pipeline
// create_default_transform, :17-33) applied to a whole batch in one launch:
//
//   dp = raw.astype(float64)                      data_module.py:132
//   ToPILImage:  u8 = uint8(dp * 255)             torchvision 0.21 to_pil_image, float ndarray
//                                                 -> (npimg * 255).astype(np.uint8): truncation
//   Grayscale:   identity on an "L" image
//   CenterCrop(image_size):                       torchvision center_crop: zero-pad a too-small
//                                                 axis by ((c-s)//2, (c-s+1)//2), else offset
//                                                 round((s-c)/2) (Python round: half to even)
//   ToTensor:    float32(u8) / 255                (1, h, w)
//
// Values outside [0, 1] are clamped before the uint8 cast (numpy's out-of-range float->uint8
// cast is platform-defined); NaN maps to 0.  HBM-bound: one thread per output pixel, reads
// the source pixel once (8 B for float64), writes 4 B.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

// torchvision center_crop source offset along one axis (negative = leading zero padding)
static int crop_offset(int size, int crop) {
  if (crop > size) return -((crop - size) / 2);
  const int d = size - crop;             // round(d / 2.0), ties to even
  const int h = d / 2;
  if ((d & 1) == 0) return h;
  return (h & 1) == 0 ? h : h + 1;
}

template <typename T>
__global__ __launch_bounds__(256) void ingest_kernel(const T* __restrict__ src, int H0, int W0,
                                                     int oh, int ow, int top, int left,
                                                     long long n, float* __restrict__ dst) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int x = (int)(i % ow);
  const long long r = i / ow;
  const int y = (int)(r % oh);
  const long long b = r / oh;
  const int sy = y + top, sx = x + left;
  float out = 0.f;
  if (sy >= 0 && sy < H0 && sx >= 0 && sx < W0) {
    const double v = (double)src[(b * H0 + sy) * W0 + sx] * 255.0;
    const double c = v > 255.0 ? 255.0 : (v > 0.0 ? v : 0.0);   // NaN -> 0
    const int u8 = (int)c;                                        // truncation, as astype
    out = (float)u8 / 255.0f;
  }
  dst[i] = out;
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_ingest_patterns(const void* src, int src_dtype, int B, int H0, int W0,
                                       int out_h, int out_w, float* dst, ebsdvae_stream_t stream) {
  EV_REQUIRE(src && dst && B >= 0 && H0 > 0 && W0 > 0 && out_h > 0 && out_w > 0,
             "ingest_patterns: bad args");
  EV_REQUIRE(src_dtype == 0 || src_dtype == 1, "ingest_patterns: src_dtype %d (0 f64, 1 f32)", src_dtype);
  if (B == 0) return 0;
  const long long n = (long long)B * out_h * out_w;
  const int top = crop_offset(H0, out_h), left = crop_offset(W0, out_w);
  const dim3 grid((unsigned)((n + 255) / 256));
  if (src_dtype == 0)
    hipLaunchKernelGGL(ingest_kernel<double>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const double*)src, H0, W0, out_h, out_w, top, left, n, dst);
  else
    hipLaunchKernelGGL(ingest_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const float*)src, H0, W0, out_h, out_w, top, left, n, dst);
  return evh::check_launch("ingest_patterns");
}
