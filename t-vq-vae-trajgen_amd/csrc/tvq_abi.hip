// ABI plumbing: thread-local error string and version.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>

#include "tvq_common.h"

namespace tvq {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

bool g_plan_trace = false;
static std::mutex g_plan_mu;
static std::string g_plan_log;
void plan_note_impl(const char* fmt, ...) {
  char line[160];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(line, sizeof(line), fmt, ap);
  va_end(ap);
  std::lock_guard<std::mutex> lock(g_plan_mu);
  if (g_plan_log.size() < (1u << 20)) {
    g_plan_log += line;
    g_plan_log += '\n';
  }
}

namespace {
// Eager launches take slots round robin from [0, lo); slots handed out while a hipGraph
// is being captured (tvq_counter_capture) come from the top of the pool, [lo, n), and are
// never handed out again: a captured graph keeps its slots for every replay, so the
// eager cursor (or another capture) must never share one with a live graph node.
struct CounterPool {
  int* base = nullptr;
  int64_t n = 0, cur = 0, lo = 0;
};
int g_capture_depth = 0;
constexpr int kMaxDevices = 64;
CounterPool g_pools[kMaxDevices];
std::mutex g_pool_mu;
// The finish classes done in-launch: norm and reduce.  Split-K slabs (gemm, conv)
// finished by one block per tile measured slower than the separate all-CU finishing
// launch, so they keep it (round 4/5 A/B; the switch was retired in round 6).
bool fused_finish_enabled(FinishClass cls) {
  static const unsigned mask = [] {
    return (1u << FIN_NORM) | (1u << FIN_REDUCE);
  }();
  return (mask >> cls) & 1u;
}
}  // namespace

int* counters(int64_t k, FinishClass cls) {
  if (k <= 0 || !fused_finish_enabled(cls)) return nullptr;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lock(g_pool_mu);
  CounterPool& p = g_pools[dev];
  if (!p.base) return nullptr;
  if (g_capture_depth > 0) {  // pinned for the graph's lifetime
    if (p.lo - k < p.n / 2) return nullptr;  // keep half the pool for eager launches
    p.lo -= k;
    if (p.cur > p.lo) p.cur = 0;
    return p.base + p.lo;
  }
  if (k > p.lo) return nullptr;  // the caller falls back to a separate finishing launch
  if (p.cur + k > p.lo) p.cur = 0;
  int* r = p.base + p.cur;
  p.cur += k;
  return r;
}
}  // namespace tvq

extern "C" int tvq_counter_capture(int64_t begin) {
  std::lock_guard<std::mutex> lock(tvq::g_pool_mu);
  tvq::g_capture_depth += begin ? 1 : -1;
  if (tvq::g_capture_depth < 0) tvq::g_capture_depth = 0;
  return TVQ_OK;
}

extern "C" int tvq_counter_pool(int64_t device, int32_t* zeroed, int64_t n) {
  TVQ_CHECK_ARG(device >= 0 && device < tvq::kMaxDevices && (zeroed || n == 0) && n >= 0,
                "tvq_counter_pool: bad arguments");
  std::lock_guard<std::mutex> lock(tvq::g_pool_mu);
  tvq::g_pools[device].base = zeroed;
  tvq::g_pools[device].n = n;
  tvq::g_pools[device].cur = 0;
  tvq::g_pools[device].lo = n;
  return TVQ_OK;
}

extern "C" int tvq_plan_trace(int64_t on) {
  std::lock_guard<std::mutex> lock(tvq::g_plan_mu);
  tvq::g_plan_log.clear();
  tvq::g_plan_trace = on != 0;
  return TVQ_OK;
}

extern "C" int64_t tvq_plan_read(char* buf, int64_t cap) {
  std::lock_guard<std::mutex> lock(tvq::g_plan_mu);
  const int64_t n = (int64_t)tvq::g_plan_log.size();
  if (buf && cap > 0) {
    const int64_t m = n < cap - 1 ? n : cap - 1;
    memcpy(buf, tvq::g_plan_log.data(), (size_t)m);
    buf[m] = 0;
  }
  return n;
}

extern "C" const char* tvq_last_error(void) { return tvq::g_err; }
extern "C" int tvq_abi_version(void) { return 1; }
