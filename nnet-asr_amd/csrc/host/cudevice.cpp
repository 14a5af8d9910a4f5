// cudevice.cpp -- see cudevice.h.
#include "cudevice.h"

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <iomanip>
#include <iostream>
#include <sstream>

namespace TNet {

// TNET_SEGV_TRACE=1: a host SIGSEGV / SIGABRT prints the faulting thread's native backtrace to stderr
// before the default action (diagnostics for crashes inside the runtime or a profiler tool, where no
// debugger may attach; the frames are resolved offline with addr2line / llvm-symbolizer).
static void segv_trace(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "\n*** tnet: fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static void install_segv_trace() {
  static bool done = false;
  if (done) return;
  done = true;
  const char* e = getenv("TNET_SEGV_TRACE");
  if (!e || e[0] != '1') return;
  signal(SIGSEGV, segv_trace);
  signal(SIGBUS, segv_trace);
  signal(SIGABRT, segv_trace);
}

CuDevice& CuDevice::Instantiate() {
  static CuDevice dev;
  dev.EnsureInit();
  return dev;
}

CuDevice::CuDevice() {}

void CuDevice::EnsureInit() {
  if (mInit) return;
  install_segv_trace();
  int n = 0;
  TNET_HIP_CALL(hipGetDeviceCount(&n));
  if (n <= 0) Error("CuDevice: no HIP device visible");
  TNET_HIP_CALL(hipSetDevice(mDevice));
  TNET_HIP_CALL(hipStreamCreateWithFlags(&mStream, hipStreamNonBlocking));
  mOwnStream = true;
  mInit = true;
}

void CuDevice::SelectGPU(int gpu_id) {
  if (!mFree.empty() || mWs) Error("CuDevice::SelectGPU after allocation");
  int n = 0;
  TNET_HIP_CALL(hipGetDeviceCount(&n));
  if (gpu_id < 0 || gpu_id >= n) Error("CuDevice::SelectGPU: invalid gpu id");
  if (mOwnStream && mStream) (void)hipStreamDestroy(mStream);
  mDevice = gpu_id;
  TNET_HIP_CALL(hipSetDevice(mDevice));
  TNET_HIP_CALL(hipStreamCreateWithFlags(&mStream, hipStreamNonBlocking));
  mOwnStream = true;
}

void CuDevice::SetStream(hipStream_t s) {
  if (mOwnStream && mStream) TNET_HIP_CALL(hipStreamSynchronize(mStream));
  if (mOwnStream && mStream) (void)hipStreamDestroy(mStream);
  mStream = s;
  mOwnStream = false;
}

void CuDevice::AccuProfile(const std::string& key, double msec) { mProfileMap[key] += msec; }

void CuDevice::PrintProfile(std::ostream& os) {
  os << "== PROFILE ==\n";
  for (auto& kv : mProfileMap) os << std::setw(24) << kv.first << " " << kv.second / 1000.0 << "\n";
  os << "=============\n";
}

void* CuDevice::Alloc(size_t bytes) {
  if (bytes == 0) return nullptr;
  auto it = mFree.find(bytes);
  if (it != mFree.end() && !it->second.empty()) {
    void* p = it->second.back();
    it->second.pop_back();
    return p;
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    // release the cache and retry once
    TNET_HIP_CALL(hipStreamSynchronize(mStream));
    for (auto& kv : mFree)
      for (void* q : kv.second) (void)hipFree(q);
    mFree.clear();
    TNET_HIP_CALL(hipMalloc(&p, bytes));
  }
  return p;
}

void CuDevice::Free(void* p, size_t bytes) {
  if (!p) return;
  mFree[bytes].push_back(p);  // stream-ordered reuse: all library work is on mStream
}

void* CuDevice::Workspace(size_t bytes) {
  if (bytes > mWsBytes) {
    if (mWs) {
      TNET_HIP_CALL(hipStreamSynchronize(mStream));
      (void)hipFree(mWs);
    }
    size_t b = bytes < (1u << 20) ? (1u << 20) : bytes;
    TNET_HIP_CALL(hipMalloc(&mWs, b));
    mWsBytes = b;
  }
  return mWs;
}

void CuDevice::Synchronize() { TNET_HIP_CALL(hipStreamSynchronize(mStream)); }

CuDevice::~CuDevice() {
  // process teardown: the HIP runtime may already be gone; do not throw
  if (!mInit) return;
  (void)hipStreamSynchronize(mStream);
  for (auto& kv : mFree)
    for (void* q : kv.second) (void)hipFree(q);
  if (mWs) (void)hipFree(mWs);
  if (mOwnStream && mStream) (void)hipStreamDestroy(mStream);
  if (mVerbose) PrintProfile(std::cout);
}

hipEvent_t CuDevice::KTEvent() {
  if (mKTNext >= mKTPool.size()) {
    hipEvent_t e;
    // timing only (no host inspection of the kernels' memory): without HIP's system-scope fence, whose L2
    // write-back + invalidate at every record would slow the timed kernels (and start them cold) in a way the
    // untimed step does not see
    TNET_HIP_CALL(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    mKTPool.push_back(e);
  }
  return mKTPool[mKTNext++];
}

void CuDevice::KTRecord(const std::string& tag, double work, hipEvent_t a, hipEvent_t b, int count) {
  mKT.push_back(KTRec{tag, work, a, b, count});
}

void CuDevice::KTRunBegin() {
  if (mKTRunOpen) return;
  KTRun r;
  r.a = KTEvent();
  TNET_HIP_CALL(hipEventRecord(r.a, mStream));
  mKTRunList.push_back(r);
  mKTRunOpen = true;
}

void CuDevice::KTRunAdd(const std::string& tag, double work, int count) {
  if (!mKTRunOpen) return;
  auto& t = mKTRunList.back().tags[tag];
  t.first += count;
  t.second += work;
}

void CuDevice::KTCloseRun() {
  if (!mKTRunOpen) return;
  mKTRunList.back().b = KTEvent();
  TNET_HIP_CALL(hipEventRecord(mKTRunList.back().b, mStream));
  mKTRunOpen = false;
}

std::string CuDevice::KTCollect() {
  KTCloseRun();
  TNET_HIP_CALL(hipStreamSynchronize(mStream));
  struct Agg {
    long n = 0;
    double ms = 0, work = 0;
  };
  std::map<std::string, Agg> agg;
  for (auto& r : mKT) {
    float ms = 0.f;
    TNET_HIP_CALL(hipEventElapsedTime(&ms, r.a, r.b));
    Agg& g = agg[r.tag];
    g.n += r.count;
    g.ms += ms;
    g.work += r.work;
  }
  Agg runs;
  long nruns = 0;
  for (auto& r : mKTRunList) {
    float ms = 0.f;
    TNET_HIP_CALL(hipEventElapsedTime(&ms, r.a, r.b));
    double work = 0;
    for (auto& t : r.tags) work += t.second.second;
    for (auto& t : r.tags) {
      Agg& g = agg[t.first];
      g.n += t.second.first;
      g.ms += work > 0 ? ms * t.second.second / work : 0.0;
      g.work += t.second.second;
      runs.n += t.second.first;
    }
    runs.ms += ms;
    runs.work += work;
    nruns++;
  }
  mKT.clear();
  mKTRunList.clear();
  mKTNext = 0;
  std::ostringstream os;
  os.precision(10);
  for (auto& kv : agg) os << kv.first << " " << kv.second.n << " " << kv.second.ms << " " << kv.second.work << "\n";
  if (nruns) os << "@runs:" << nruns << " " << runs.n << " " << runs.ms << " " << runs.work << "\n";
  return os.str();
}

KTScope::KTScope(const std::string& tag, double work, int count) : mTag(tag), mWork(work), mCount(count) {
  CuDevice& d = CuDevice::Instantiate();
  if (!d.KernelTiming()) return;
  if (d.KernelTimingRuns()) {
    if (d.KernelTimed(tag)) {
      d.KTRunBegin();
      mRun = true;
    } else {
      d.KTCloseRun();
    }
    return;
  }
  if (!d.KernelTimed(tag)) return;
  mA = d.KTEvent();
  TNET_HIP_CALL(hipEventRecord(mA, d.Stream()));
}

KTScope::~KTScope() {
  CuDevice& d = CuDevice::Instantiate();
  if (mRun) {
    d.KTRunAdd(mTag, mWork, mCount);
    return;
  }
  if (!mA) return;
  hipEvent_t b = d.KTEvent();
  (void)hipEventRecord(b, d.Stream());
  d.KTRecord(mTag, mWork, mA, b, mCount);
}

CuProfileScope::CuProfileScope(const char* key) : mKey(key) {
  CuDevice& d = CuDevice::Instantiate();
  if (!d.Profile()) return;
  (void)hipEventCreate(&mStart);
  (void)hipEventCreate(&mStop);
  (void)hipEventRecord(mStart, d.Stream());
}

CuProfileScope::~CuProfileScope() {
  if (!mStart) return;
  CuDevice& d = CuDevice::Instantiate();
  (void)hipEventRecord(mStop, d.Stream());
  (void)hipEventSynchronize(mStop);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, mStart, mStop);
  d.AccuProfile(mKey, ms);
  (void)hipEventDestroy(mStart);
  (void)hipEventDestroy(mStop);
}

}  // namespace TNet
