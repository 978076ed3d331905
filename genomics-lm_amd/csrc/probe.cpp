// Live kernel probe: HIP events recorded on the launching stream around every launch of
// one selected kernel, plus that launch's algorithmic work (FLOPs or bytes).  bench.py
// turns it on for the timed region and reads back (work, device ms, launches) to report
// the dominant kernel's roofline from the real step, not from a replay.
#include <hip/hip_runtime.h>
#include <mutex>
#include <vector>
#include "../../include/codonlm_hip.h"
#include "probe.h"

namespace {
struct Probe {
  int kind = 0;
  std::vector<hipEvent_t> pool;  // pairs: start, stop
  size_t used = 0;
  double work = 0.0;
  double bytes = 0.0;   // algorithmic HBM bytes of the recorded launches (operands once + outputs once)
  long long launches = 0;
  long long seen = 0;   // launches of the selected kernel since enable
  int every = 1;        // record 1 of every `every` launches (sampling keeps the event cost low)
  bool open = false;    // the current launch is being recorded
  std::mutex mu;
} g_probe;
}  // namespace

int cg_probe_kind() { return g_probe.kind; }

void cg_probe_begin(int kind, hipStream_t s) {
  if (g_probe.kind != kind) return;
  std::lock_guard<std::mutex> lk(g_probe.mu);
  g_probe.open = (g_probe.seen++ % g_probe.every) == 0;
  if (!g_probe.open) return;
  if (g_probe.used + 2 > g_probe.pool.size()) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) {
        g_probe.open = false;
        return;
      }
      g_probe.pool.push_back(e);
    }
  }
  (void)hipEventRecord(g_probe.pool[g_probe.used], s);
}

void cg_probe_end(int kind, hipStream_t s, double work, double bytes) {
  if (g_probe.kind != kind) return;
  std::lock_guard<std::mutex> lk(g_probe.mu);
  if (!g_probe.open) return;
  g_probe.open = false;
  (void)hipEventRecord(g_probe.pool[g_probe.used + 1], s);
  g_probe.used += 2;
  g_probe.work += work;
  g_probe.bytes += bytes;
  g_probe.launches += 1;
}

extern "C" int cg_probe_enable(int kind) {
  std::lock_guard<std::mutex> lk(g_probe.mu);
  g_probe.kind = kind;
  g_probe.used = 0;
  g_probe.work = 0.0;
  g_probe.bytes = 0.0;
  g_probe.launches = 0;
  g_probe.seen = 0;
  g_probe.open = false;
  return CG_OK;
}

extern "C" int cg_probe_sample(int every) {
  if (every < 1) return CG_EINVAL;
  std::lock_guard<std::mutex> lk(g_probe.mu);
  g_probe.every = every;
  return CG_OK;
}

// synchronises on the recorded events; returns total device ms over the probed launches
extern "C" int cg_probe_read(double* work, double* ms, long long* launches) {
  std::lock_guard<std::mutex> lk(g_probe.mu);
  double tot = 0.0;
  for (size_t i = 0; i + 1 < g_probe.used; i += 2) {
    if (hipEventSynchronize(g_probe.pool[i + 1]) != hipSuccess) return CG_ELAUNCH;
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_probe.pool[i], g_probe.pool[i + 1]) != hipSuccess) return CG_ELAUNCH;
    tot += t;
  }
  if (work) *work = g_probe.work;
  if (ms) *ms = tot;
  if (launches) *launches = g_probe.launches;
  return CG_OK;
}

extern "C" int cg_probe_bytes(double* bytes) {
  std::lock_guard<std::mutex> lk(g_probe.mu);
  if (bytes) *bytes = g_probe.bytes;
  return CG_OK;
}
