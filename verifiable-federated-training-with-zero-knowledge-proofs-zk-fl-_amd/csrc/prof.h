// Per-kernel HIP-event timing on the context stream (bench.py roofline: the dominant
// kernel's average launch duration is measured live on the stream it is launched on).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

namespace zkfl {

struct ProfRec {
  std::string name;
  hipEvent_t a = nullptr, b = nullptr;
  double units = 0;          // algorithmic units known on the host
  uint32_t* units_dev = nullptr;  // or counted on the device (read after sync)
};

struct Profiler {
  bool on = false;
  bool serialize = false;  // run every proof stream on the slot's main stream (isolated kernel timings)
  std::vector<ProfRec> recs;
  std::vector<uint32_t*> dev_counters;  // pinned host slots for device-counted units

  int begin(const char* name, hipStream_t st) {
    if (!on) return -1;
    ProfRec r;
    r.name = name;
    (void)hipEventCreate(&r.a);
    (void)hipEventCreate(&r.b);
    (void)hipEventRecord(r.a, st);
    recs.push_back(r);
    return (int)recs.size() - 1;
  }
  // d_units: optional device uint32 counter copied after the launch
  void end(int idx, hipStream_t st, double units, const uint32_t* d_units = nullptr) {
    if (idx < 0) return;
    ProfRec& r = recs[idx];
    (void)hipEventRecord(r.b, st);
    r.units = units;
    if (d_units) {
      uint32_t* h = nullptr;
      if (hipHostMalloc(&h, sizeof(uint32_t)) == hipSuccess) {
        (void)hipMemcpyAsync(h, d_units, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
        r.units_dev = h;
      }
    }
  }
  void reset() {
    for (auto& r : recs) {
      if (r.a) (void)hipEventDestroy(r.a);
      if (r.b) (void)hipEventDestroy(r.b);
      if (r.units_dev) (void)hipHostFree(r.units_dev);
    }
    recs.clear();
  }
  // Sum (and median launch time) over records with this name.  Caller synchronises first.
  void query(const std::string& name, double* ms, uint64_t* launches, double* units, double* median_ms) {
    double t = 0, u = 0;
    std::vector<double> d;
    for (auto& r : recs) {
      if (r.name != name) continue;
      float e = 0;
      if (hipEventElapsedTime(&e, r.a, r.b) == hipSuccess) t += e;
      d.push_back(e);
      u += r.units_dev ? (double)*r.units_dev : r.units;
    }
    *ms = t;
    *launches = d.size();
    if (units) *units = u;
    if (median_ms) {
      std::sort(d.begin(), d.end());
      *median_ms = d.empty() ? 0.0 : (d.size() & 1 ? d[d.size() / 2] : 0.5 * (d[d.size() / 2 - 1] + d[d.size() / 2]));
    }
  }
};

}  // namespace zkfl
