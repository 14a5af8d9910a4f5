// cudevice.h -- per-process device context of the MI355X TNet library.
//
// Counterpart of CuDevice (src/CuBaseLib/cudevice.h:15-73, cudevice.cc:23-121): GPU selection,
// verbose/profile map (AccuProfile).  Differences, MI355X-first:
//   * created lazily on first use (the reference builds it at static-init time, cudevice.cc:121),
//     so loading the library never touches the GPU;
//   * owns one HIP stream on which every operation of the library is enqueued asynchronously
//     (no per-call device sync); host values are only read back where the API demands them;
//   * owns a size-bucketed caching allocator (steady-state training performs no hipMalloc) and
//     the stream-ordered scratch workspace the reduction kernels need;
//   * profiling: when enabled, ops are bracketed by hipEvents and accumulated per name, the
//     AccuProfile map of the reference (printed by PrintProfile).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "tnet_common.h"

namespace TNet {

class CuDevice {
 public:
  static CuDevice& Instantiate();

  hipStream_t Stream() { return mStream; }
  /// Use an external stream (e.g. a caller-owned one); the library does not destroy it.
  void SetStream(hipStream_t s);
  int DeviceId() const { return mDevice; }
  /// SelectGPU (cudevice.cc:84-101): must be called before any allocation.
  void SelectGPU(int gpu_id);

  void Verbose(bool v) { mVerbose = v; }
  bool Verbose() const { return mVerbose; }
  void Profile(bool p) { mProfile = p; }
  bool Profile() const { return mProfile; }
  void AccuProfile(const std::string& key, double msec);
  void PrintProfile(std::ostream& os);
  const std::map<std::string, double>& ProfileMap() const { return mProfileMap; }

  // ---- per-kernel device timing (hipEvent pairs around launches; off by default)
  /// mode 0 off; 1 an event pair around every timed launch; 2 RUNS: consecutive timed launches share
  /// one event pair (a scope whose tag fails the filter, or the report, closes the run), so a chain of
  /// back-to-back timed kernels carries one pair instead of one per launch.  A run's time is split over
  /// its tags by work share; the exact run totals are reported on a "@runs" line.
  void KernelTiming(int mode) {
    if (mode == 0) KTCloseRun();
    mKTOn = mode != 0;
    mKTRuns = mode == 2;
  }
  bool KernelTiming() const { return mKTOn; }
  bool KernelTimingRuns() const { return mKTRuns; }
  /// run mode: a timed launch begins (opens a run unless one is open)
  void KTRunBegin();
  /// run mode: a timed launch ended (its work joins the open run)
  void KTRunAdd(const std::string& tag, double work, int count = 1);
  /// run mode: an untimed launch begins / the report is taken: close the open run
  void KTCloseRun();
  /// time only the launches whose tag contains `filter` (empty = all): each event pair costs
  /// a few microseconds of stream time, so a benchmark times only the kernel it reports
  void KernelTimingFilter(const std::string& filter) { mKTFilter = filter; }
  /// the filter selects tags containing it, or -- "prefix*suffix" -- tags starting with prefix and ending
  /// with suffix ("gemm_*:2048x2048": the 2048x2048 GEMM launches, not the data-parallel applies of that
  /// shape, which run on another stream)
  bool KernelTimed(const std::string& tag) const {
    if (!mKTOn) return false;
    if (mKTFilter.empty()) return true;
    const size_t star = mKTFilter.find('*');
    if (star == std::string::npos) return tag.find(mKTFilter) != std::string::npos;
    const size_t np = star, ns = mKTFilter.size() - star - 1;
    return tag.size() >= np + ns && tag.compare(0, np, mKTFilter, 0, np) == 0 &&
           tag.compare(tag.size() - ns, ns, mKTFilter, star + 1, ns) == 0;
  }
  void KTRecord(const std::string& tag, double work, hipEvent_t a, hipEvent_t b, int count = 1);
  hipEvent_t KTEvent();
  /// sync, aggregate "tag count total_ms total_work" lines, reset
  std::string KTCollect();

  void* Alloc(size_t bytes);
  void Free(void* p, size_t bytes);
  /// Scratch buffer valid until the next Workspace() call on this stream (stream-ordered reuse).
  void* Workspace(size_t bytes);
  void Synchronize();

  ~CuDevice();

 private:
  CuDevice();
  CuDevice(const CuDevice&) = delete;
  CuDevice& operator=(const CuDevice&) = delete;
  void EnsureInit();

  bool mInit = false;
  int mDevice = 0;
  hipStream_t mStream = nullptr;
  bool mOwnStream = false;
  bool mVerbose = false;
  bool mProfile = false;
  std::map<std::string, double> mProfileMap;
  std::map<size_t, std::vector<void*>> mFree;
  void* mWs = nullptr;
  size_t mWsBytes = 0;
  bool mKTOn = false;
  bool mKTRuns = false;
  std::string mKTFilter;
  struct KTRun {
    std::map<std::string, std::pair<long, double>> tags;  // tag -> (launches, work)
    hipEvent_t a = nullptr, b = nullptr;
  };
  std::vector<KTRun> mKTRunList;
  bool mKTRunOpen = false;
  struct KTRec {
    std::string tag;
    double work;
    hipEvent_t a, b;
    int count;
  };
  std::vector<KTRec> mKT;
  std::vector<hipEvent_t> mKTPool;
  size_t mKTNext = 0;
};

/// RAII device timing of the launches enqueued in its scope (when KernelTiming is on).
class KTScope {
 public:
  /// count: the GEMMs the scope's launch carries (a paired launch counts as its two)
  KTScope(const std::string& tag, double work, int count = 1);
  ~KTScope();
  /// nothing was launched in the scope after all: record nothing
  void Cancel() {
    mRun = false;
    mA = nullptr;
  }

 private:
  std::string mTag;
  double mWork;
  int mCount;
  hipEvent_t mA = nullptr;
  bool mRun = false;
};

/// RAII profile scope: times the enqueued work of one op when profiling is on.
class CuProfileScope {
 public:
  explicit CuProfileScope(const char* key);
  ~CuProfileScope();

 private:
  const char* mKey;
  hipEvent_t mStart = nullptr, mStop = nullptr;
};

}  // namespace TNet
