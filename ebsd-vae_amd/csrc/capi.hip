// Error plumbing and version of the C ABI (include/ebsdvae.h).
#include <stdarg.h>
#include <stdio.h>

#include <mutex>

#include "common.h"
#include "../../include/ebsdvae.h"

namespace {
thread_local char g_err[512] = "";
}

namespace evh {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}
}  // namespace evh

extern "C" const char* ebsdvae_last_error(void) { return g_err; }
extern "C" int ebsdvae_version(void) { return 1; }

// ------------------------------------------------------------------ cross-stream ordering
// `waiter` waits for the work enqueued on `signaler` so far, through an event recorded with a
// device-scope release (hipEventReleaseToDevice) instead of the default system-scope fence:
// both streams run on this device, so nothing needs to become visible to the host, and the
// system-scope writeback + invalidate of every fork / join costs the GPU a few microseconds of
// idle time (tools/step_gaps.py).  A wait takes the event's state at enqueue time, so a small
// ring of events per device is reused round-robin; capturable into hipGraphs (fork / join).
// The ring is the signaler stream's device's (not the caller's current device), created
// on that device; ring creation and the round-robin index are guarded, since forward and
// autograd-backward threads both fork and join.
extern "C" int ebsdvae_stream_wait(ebsdvae_stream_t waiter, ebsdvae_stream_t signaler) {
  constexpr int kRing = 64, kMaxDev = 64;
  static hipEvent_t ring[kMaxDev][kRing];
  static int next[kMaxDev];
  static bool made[kMaxDev];
  static std::mutex mu;
  int dev = -1;
  if (signaler == nullptr || hipStreamGetDevice((hipStream_t)signaler, &dev) != hipSuccess) {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  if (dev < 0 || dev >= kMaxDev) {
    evh::set_error("stream_wait: no device for the signaler stream");
    return 2;
  }
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> lock(mu);
    if (!made[dev]) {
      int cur = 0;
      if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(dev) != hipSuccess) {
        evh::set_error("stream_wait: cannot select device %d", dev);
        return 2;
      }
      bool ok = true;
      for (int i = 0; i < kRing && ok; ++i)
        ok = hipEventCreateWithFlags(&ring[dev][i],
                                     hipEventDisableTiming | hipEventReleaseToDevice) == hipSuccess;
      (void)hipSetDevice(cur);
      if (!ok) {
        evh::set_error("stream_wait: hipEventCreateWithFlags failed");
        return 2;
      }
      made[dev] = true;
    }
    ev = ring[dev][next[dev]];
    next[dev] = (next[dev] + 1) % kRing;
  }
  if (hipEventRecord(ev, (hipStream_t)signaler) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)waiter, ev, 0) != hipSuccess) {
    evh::set_error("stream_wait: %s", hipGetErrorString(hipGetLastError()));
    return 2;
  }
  return 0;
}
