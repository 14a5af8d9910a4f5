// trainer.cpp -- see trainer.h.
#include "trainer.h"

#include <rccl/rccl.h>

#include <cstring>
#include <sys/time.h>

namespace TNet {

// ======================================================================================
// CuTrainer
// ======================================================================================
CuTrainer::CuTrainer(CuNetwork* net, CuObjectiveFunction* obj, const TrainerOptions& opt)
    : mNet(net), mObj(obj), mOpt(opt) {
  if (mOpt.bunchsize == 0) Error("CuTrainer: bunchsize must be > 0");
  // make the cachesize divisible by bunchsize (TNetCu.cc:362)
  mOpt.cachesize = (mOpt.cachesize / mOpt.bunchsize) * mOpt.bunchsize;
  if (mOpt.cachesize == 0) Error("CuTrainer: cachesize smaller than bunchsize");
  long seed = mOpt.seed;
  if (seed == 0) {
    struct timeval tv;
    gettimeofday(&tv, 0);
    seed = (int)(tv.tv_sec) + (int)tv.tv_usec;
  }
  mRng.Seed(seed);
  mCache.Init(mOpt.cachesize, mOpt.bunchsize);
  mCache.SetRng(&mRng);
  mCache.Trace(mOpt.trace);
}

CuTrainer::~CuTrainer() {}

void CuTrainer::Step() {
  mCache.GetBunchLabels(mFeats, mLabels);
  mNet->TrainBunch(mFeats, mLabels, *mObj, !mOpt.crossval, mOpt.crossval ? nullptr : mExchange);
  if (mOpt.trace & 2) std::cout << "." << std::flush;
  mSteps++;
}

void CuTrainer::DrainCache() {
  if (mOpt.randomize) mCache.Randomize();
  while (!mCache.Empty()) Step();
  mTrainedSinceFill = true;
}

void CuTrainer::AddUtterance(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels) {
  if (cols != mNet->GetNInputs()) {
    std::ostringstream os;
    os << "CuTrainer::AddUtterance: feature dim " << cols << " != network input dim " << mNet->GetNInputs();
    Error(os.str());
  }
  if (rows == 0) return;
  mCache.AddDataHost(feats, rows, cols, ld, labels);
  mTrainedSinceFill = false;
  if (mCache.Full()) DrainCache();
}

void CuTrainer::Finish() {
  // TNetCu.cc:376-441: after EndOfList the (partial) cache filled so far is drained once;
  // a leftover still pending after a full cache was drained is dropped.
  if (!mTrainedSinceFill && mCache.IntakePos() > 0) DrainCache();
  if (mExchange) {
    double v[1] = {(double)mSteps};
    double mx[1] = {v[0]};
    mExchange->AllReduceHost(mx, 1);
    if (mx[0] != v[0] * mExchange->WorldSize())
      Error("CuTrainer: data-parallel ranks took different numbers of steps (unequal shards)");
  }
}

size_t CuTrainer::Prefill(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels) {
  if (mCache.Full()) return 0;
  const size_t space = mOpt.cachesize - mCache.IntakePos();
  const size_t take = rows < space ? rows : space;
  mCache.AddDataHost(feats, take, cols, ld, labels);
  if (mCache.Full() && mOpt.randomize) mCache.Randomize();
  return take;
}

void CuTrainer::Replay(long n) {
  for (long i = 0; i < n; i++) {
    if (mCache.Empty()) {
      mCache.Rewind();
      if (mOpt.randomize) mCache.Randomize();
    }
    Step();
  }
}

// ======================================================================================
// RCCL exchange
// ======================================================================================
#define NCCL_CALL(x)                                                                    \
  do {                                                                                  \
    ncclResult_t _r = (x);                                                              \
    if (_r != ncclSuccess) {                                                            \
      std::ostringstream _os;                                                           \
      _os << "RCCL ERROR " << ncclGetErrorString(_r) << " at " << __FILE__ << ":" << __LINE__ << " '" #x "'"; \
      throw MyException(_os.str());                                                     \
    }                                                                                   \
  } while (0)

struct RcclExchange::Impl {
  ncclComm_t comm = nullptr;
  hipStream_t comm_stream = nullptr;
  std::vector<hipEvent_t> events;
  size_t next_event = 0;
  hipEvent_t done = nullptr;
  double* dscratch = nullptr;
};

void RcclExchange::UniqueId(char out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  NCCL_CALL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, 128);
}

RcclExchange::RcclExchange(int rank, int world, const char id[128]) : mImpl(new Impl), mRank(rank), mWorld(world) {
  CuDevice& dev = CuDevice::Instantiate();
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  NCCL_CALL(ncclCommInitRank(&mImpl->comm, world, uid, rank));
  TNET_HIP_CALL(hipStreamCreateWithFlags(&mImpl->comm_stream, hipStreamNonBlocking));
  TNET_HIP_CALL(hipEventCreateWithFlags(&mImpl->done, hipEventDisableTiming));
  TNET_HIP_CALL(hipMalloc(&mImpl->dscratch, 4096));
  (void)dev;
}

RcclExchange::~RcclExchange() {
  if (!mImpl) return;
  (void)hipStreamSynchronize(mImpl->comm_stream);
  for (auto e : mImpl->events) (void)hipEventDestroy(e);
  if (mImpl->done) (void)hipEventDestroy(mImpl->done);
  if (mImpl->dscratch) (void)hipFree(mImpl->dscratch);
  if (mImpl->comm) (void)ncclCommDestroy(mImpl->comm);
  if (mImpl->comm_stream) (void)hipStreamDestroy(mImpl->comm_stream);
}

void RcclExchange::Submit(CuUpdatableComponent& comp) {
  CuDevice& dev = CuDevice::Instantiate();
  if (mImpl->next_event >= mImpl->events.size()) {
    hipEvent_t e;
    TNET_HIP_CALL(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    mImpl->events.push_back(e);
  }
  hipEvent_t ev = mImpl->events[mImpl->next_event++];
  // the gradient kernels were enqueued on the compute stream: order the reduction after them
  TNET_HIP_CALL(hipEventRecord(ev, dev.Stream()));
  TNET_HIP_CALL(hipStreamWaitEvent(mImpl->comm_stream, ev, 0));
  std::vector<CuParamBlock> blocks = comp.GradientBlocks();
  NCCL_CALL(ncclGroupStart());
  for (auto& b : blocks)
    NCCL_CALL(ncclAllReduce(b.grad, b.grad, (size_t)b.n, ncclFloat, ncclSum, mImpl->comm, mImpl->comm_stream));
  NCCL_CALL(ncclGroupEnd());
}

void RcclExchange::WaitAll() {
  CuDevice& dev = CuDevice::Instantiate();
  TNET_HIP_CALL(hipEventRecord(mImpl->done, mImpl->comm_stream));
  TNET_HIP_CALL(hipStreamWaitEvent(dev.Stream(), mImpl->done, 0));
  mImpl->next_event = 0;
}

void RcclExchange::AllReduceHost(double* v, int n) {
  if (n <= 0) return;
  if (n > 512) Error("RcclExchange::AllReduceHost: too many values");
  CuDevice& dev = CuDevice::Instantiate();
  TNET_HIP_CALL(hipStreamSynchronize(dev.Stream()));
  TNET_HIP_CALL(hipMemcpyAsync(mImpl->dscratch, v, n * sizeof(double), hipMemcpyHostToDevice, mImpl->comm_stream));
  NCCL_CALL(ncclAllReduce(mImpl->dscratch, mImpl->dscratch, n, ncclDouble, ncclSum, mImpl->comm, mImpl->comm_stream));
  TNET_HIP_CALL(hipMemcpyAsync(v, mImpl->dscratch, n * sizeof(double), hipMemcpyDeviceToHost, mImpl->comm_stream));
  TNET_HIP_CALL(hipStreamSynchronize(mImpl->comm_stream));
}

void RcclExchange::AllReduceDevice(float* buf, size_t n) {
  CuDevice& dev = CuDevice::Instantiate();
  TNET_HIP_CALL(hipStreamSynchronize(dev.Stream()));
  NCCL_CALL(ncclAllReduce(buf, buf, n, ncclFloat, ncclSum, mImpl->comm, mImpl->comm_stream));
  TNET_HIP_CALL(hipStreamSynchronize(mImpl->comm_stream));
}

}  // namespace TNet
