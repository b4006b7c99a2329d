// Error plumbing and version of the C ABI (include/ebsdvae.h).
#include <stdarg.h>
#include <stdio.h>

#include <mutex>
#include <vector>

#include <hip/hip_ext.h>

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
// ABI version (include/ebsdvae.h EBSDVAE_ABI_VERSION): 2 since the heads entry points took
// their caller-owned `work` scratch (round 4); latice/_native.load() refuses any other value
extern "C" int ebsdvae_version(void) { return EBSDVAE_ABI_VERSION; }

// ------------------------------------------------------------------ cross-stream ordering
// `waiter` waits for the work enqueued on `signaler` so far, through an event recorded with the
// default system-scope release (round 6; EBSDVAE_FORK_DEVICE_SCOPE=1 selects the device-scope
// release, hipEventReleaseToDevice, used through round 5: the same step time either way, and the
// system scope takes the one non-default synchronisation choice off the side-stream path whose
// single unexplained stale read DESIGN.md section 13 records).  A wait takes the event's state at
// enqueue time, so a small
// ring of events per device is reused round-robin; capturable into hipGraphs (fork / join).
// The ring is the signaler stream's device's (not the caller's current device), created
// on that device; ring creation and the round-robin index are guarded, since forward and
// autograd-backward threads both fork and join.
namespace {
// ring[kind][device]: kind 0 = fork / join events (no timing), kind 1 =
// kernel-attached fork events (signalled by the completion of the launch they are attached to)
constexpr int kRing = 64, kMaxDev = 64;
hipEvent_t g_ring[2][kMaxDev][kRing];
int g_next[2][kMaxDev];
bool g_made[2][kMaxDev];
std::mutex g_mu;

// the next event of the signaler stream's device's ring `kind` (created on first use)
int ring_event(ebsdvae_stream_t signaler, int kind, hipEvent_t* out) {
  int dev = -1;
  if (signaler == nullptr || hipStreamGetDevice((hipStream_t)signaler, &dev) != hipSuccess) {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  if (dev < 0 || dev >= kMaxDev) {
    evh::set_error("stream_wait: no device for the signaler stream");
    return 2;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_made[kind][dev]) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || hipSetDevice(dev) != hipSuccess) {
      evh::set_error("stream_wait: cannot select device %d", dev);
      return 2;
    }
    bool ok = true;
    const char* ds = getenv("EBSDVAE_FORK_DEVICE_SCOPE");
    const unsigned f0 = hipEventDisableTiming | ((ds && ds[0] == '1') ? hipEventReleaseToDevice : 0u);
    for (int i = 0; i < kRing && ok; ++i)
      ok = hipEventCreateWithFlags(&g_ring[kind][dev][i], kind == 0 ? f0 : hipEventDefault) == hipSuccess;
    (void)hipSetDevice(cur);
    if (!ok) {
      evh::set_error("stream_wait: hipEventCreateWithFlags failed");
      return 2;
    }
    g_made[kind][dev] = true;
  }
  *out = g_ring[kind][dev][g_next[kind][dev]];
  g_next[kind][dev] = (g_next[kind][dev] + 1) % kRing;
  return 0;
}

// kernel-attached fork (ebsdvae_fork_arm / ebsdvae_fork_wait), per host thread: the forward and
// the autograd backward threads each arm and consume their own
thread_local hipEvent_t g_fork_ev = nullptr;
thread_local int g_fork_state = 0;   // 0 none, 1 armed, 2 attached to a launch
}  // namespace

namespace evh {
hipEvent_t take_fork_event() {
  if (g_fork_state != 1) return nullptr;
  g_fork_state = 2;
  return g_fork_ev;
}
}  // namespace evh

extern "C" int ebsdvae_stream_wait(ebsdvae_stream_t waiter, ebsdvae_stream_t signaler) {
  hipEvent_t ev;
  if (ring_event(signaler, 0, &ev)) return 2;
  if (hipEventRecord(ev, (hipStream_t)signaler) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)waiter, ev, 0) != hipSuccess) {
    evh::set_error("stream_wait: %s", hipGetErrorString(hipGetLastError()));
    return 2;
  }
  return 0;
}

// Fork without an event record on the signaler: the next launch of the InstanceNorm-backward
// apply (the kernel that produces the weight gradient's gy) carries an event that its own
// completion signals (hipExtLaunchKernel stopEvent), and ebsdvae_fork_wait makes the waiter
// wait on it.  A record packet on the main stream between the apply and the input-gradient
// conv left the GPU idle for ~7 us per fork (tools/step_gaps.py).
extern "C" int ebsdvae_fork_arm(ebsdvae_stream_t signaler) {
  hipEvent_t ev;
  if (ring_event(signaler, 1, &ev)) return 2;
  g_fork_ev = ev;
  g_fork_state = 1;
  return 0;
}

// `waiter` waits for the armed launch if one took the event; otherwise (nothing launched since
// the arm) it falls back to ebsdvae_stream_wait on `signaler`.  Disarms either way.
extern "C" int ebsdvae_fork_wait(ebsdvae_stream_t waiter, ebsdvae_stream_t signaler) {
  const int st = g_fork_state;
  g_fork_state = 0;
  if (st != 2) return ebsdvae_stream_wait(waiter, signaler);
  if (hipStreamWaitEvent((hipStream_t)waiter, g_fork_ev, 0) != hipSuccess) {
    evh::set_error("fork_wait: %s", hipGetErrorString(hipGetLastError()));
    return 2;
  }
  return 0;
}

// ------------------------------------------------------------------ CU-partitioned streams
// A stream restricted to the CU-mask bits [first, first + count) (hipExtStreamCreateWithCUMask).
// On MI355X the runtime spreads N contiguous mask bits evenly over the 8 XCDs (N / 8 CUs each;
// tools/micro/cumask_probe.hip), so complementary ranges give two disjoint CU sets with the same
// share of every XCD.  The count is registered for the stream: the persistent conv kernels
// launched on it size their grids by it (one block per CU of the set).  Round-5 experiment of
// the CU-partitioned backward: input-gradient chain on one set, weight
// gradients on the other.
namespace {
constexpr int kMaxCuStreams = 16;
hipStream_t g_cu_stream[kMaxCuStreams];
int g_cu_count[kMaxCuStreams];
std::mutex g_cu_mu;
}  // namespace

namespace evh {
int stream_cus(hipStream_t s) {
  if (!s) return 0;
  std::lock_guard<std::mutex> lock(g_cu_mu);
  for (int i = 0; i < kMaxCuStreams; ++i)
    if (g_cu_stream[i] == s) return g_cu_count[i];
  return 0;
}
}  // namespace evh

extern "C" int ebsdvae_stream_create_cus(int first, int count, ebsdvae_stream_t* out) {
  int ncu = 0, dev = 0;
  EV_REQUIRE(out != nullptr, "stream_create_cus: null output");
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    evh::set_error("stream_create_cus: no device");
    return 2;
  }
  EV_REQUIRE(first >= 0 && count > 0 && first + count <= ncu && count % 8 == 0,
             "stream_create_cus: CUs [%d, %d) outside [0, %d) or not a multiple of 8", first,
             first + count, ncu);
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int i = first; i < first + count; ++i) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
    evh::set_error("stream_create_cus: hipExtStreamCreateWithCUMask failed");
    return 2;
  }
  std::lock_guard<std::mutex> lock(g_cu_mu);
  for (int i = 0; i < kMaxCuStreams; ++i)
    if (!g_cu_stream[i]) {
      g_cu_stream[i] = s;
      g_cu_count[i] = count;
      *out = (ebsdvae_stream_t)s;
      return 0;
    }
  (void)hipStreamDestroy(s);
  evh::set_error("stream_create_cus: more than %d CU-masked streams", kMaxCuStreams);
  return 2;
}

extern "C" int ebsdvae_stream_destroy_cus(ebsdvae_stream_t stream) {
  std::lock_guard<std::mutex> lock(g_cu_mu);
  for (int i = 0; i < kMaxCuStreams; ++i)
    if (g_cu_stream[i] == (hipStream_t)stream) {
      g_cu_stream[i] = nullptr;
      g_cu_count[i] = 0;
      return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? 0 : 2;
    }
  evh::set_error("stream_destroy_cus: not a stream of ebsdvae_stream_create_cus");
  return 1;
}
