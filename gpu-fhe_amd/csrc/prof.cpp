// Optional per-launch timing marks (used by bench.py to time individual kernels with HIP events
// on the launch stream).  Off unless fhe_prof_begin() was called on this host thread.
#include <cstring>
#include <vector>

#include "../../include/fhecore.h"
#include "internal.hpp"

namespace fhe {
namespace {
struct Recorder {
  bool on = false;
  std::vector<hipEvent_t> ev;  // ev[0] = begin, ev[i] = after launch i
  std::vector<const char*> names;
  size_t used = 0;
};
thread_local Recorder g_rec;
}  // namespace

void prof_mark(hipStream_t s, const char* name) {
  Recorder& r = g_rec;
  if (!r.on || r.used >= r.ev.size()) return;
  (void)hipEventRecord(r.ev[r.used], s);
  r.names[r.used] = name;
  ++r.used;
}

}  // namespace fhe

using namespace fhe;

extern "C" {

int fhe_prof_begin(uint32_t max_marks, fhe_stream_t stream) {
  Recorder& r = g_rec;
  if (r.ev.size() < (size_t)max_marks + 1) {
    for (auto e : r.ev) (void)hipEventDestroy(e);
    r.ev.assign(max_marks + 1, nullptr);
    // timing-only marks: without the system-scope fence a record costs no L2 writeback /
    // invalidate, which would otherwise add ~6 us of idle GPU at every mark (rocprofv3 trace)
    for (auto& e : r.ev) FHE_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  }
  r.names.assign(r.ev.size(), "");
  r.used = 0;
  r.on = true;
  prof_mark(static_cast<hipStream_t>(stream), "begin");
  return kOk;
}

int fhe_prof_end(float* elapsed_ms, uint32_t cap, uint32_t* count, char* names, size_t names_cap) {
  Recorder& r = g_rec;
  r.on = false;
  if (r.used == 0) {
    *count = 0;
    return kOk;
  }
  FHE_HIP_CHECK(hipEventSynchronize(r.ev[r.used - 1]));
  const uint32_t n = (uint32_t)std::min<size_t>(r.used - 1, cap);
  std::string all;
  for (uint32_t i = 0; i < n; ++i) {
    FHE_HIP_CHECK(hipEventElapsedTime(&elapsed_ms[i], r.ev[i], r.ev[i + 1]));
    all += r.names[i + 1];
    all += '\n';
  }
  if (names && names_cap) {
    std::strncpy(names, all.c_str(), names_cap - 1);
    names[names_cap - 1] = 0;
  }
  *count = n;
  return kOk;
}

}  // extern "C"
