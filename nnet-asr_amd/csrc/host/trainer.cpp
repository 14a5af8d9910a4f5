// trainer.cpp -- see trainer.h.
#include "trainer.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <limits>
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

// The next bunch's gather handed to the network for the step's last launch (CuNetwork::SetTailGather).
// Finish(): if no launch carried it, launch it now (checked).  If the step throws first, the destructor
// clears the network's descriptor and launches the gather unchecked, so the bunch the cache already moved
// past still lands in the other buffer and the next Step trains it.
struct TailGatherGuard {
  CuNetwork& net;
  hipStream_t stream;
  BunchGather g;
  bool armed = false;
  TailGatherGuard(CuNetwork& n, hipStream_t s) : net(n), stream(s) {}
  void Arm(const BunchGather& gather, bool ride) {
    g = gather;
    armed = true;
    if (ride) net.SetTailGather(&g);
  }
  bool Take() {
    if (!armed) return false;
    armed = false;
    const bool done = net.TailGatherDone();
    net.SetTailGather(nullptr);
    return !done;
  }
  void Finish() {
    if (!Take()) return;
    KTScope kt("gather", 2.0 * g.dy.rows * g.dy.cols * 4.0);
    TNET_SAFE_CALL(tnet_gather_bunch(g.y, g.x, g.labels_out, g.labels_in, g.copy_from, g.dy, g.dx, stream));
  }
  ~TailGatherGuard() {
    if (Take()) (void)tnet_gather_bunch(g.y, g.x, g.labels_out, g.labels_in, g.copy_from, g.dy, g.dx, stream);
  }
};

void CuTrainer::Step() {
  hipStream_t cs = CuDevice::Instantiate().Stream();
  if (mAhead) {  // gathered by the previous step's last launch, in compute-stream order (no wait)
    mCur ^= 1;
    mAhead = false;
  } else {
    mCache.GetBunchLabels(mFeatsB[mCur], mLabelsB[mCur]);
  }
  // (round 2's form, the next bunch gathered on a stream of its own beside the step, was measured slower --
  // MLP3 9.7 M vs 11.0 M frames/s, dnn4 939 k vs 952 k: the per-step cross-stream wait -- and is gone since
  // round 6; profiles/r02_* keep the A/B)
  // On by default (TNET_GATHER_TAIL=0 turns it off): the next bunch of the fill is gathered into the other
  // buffer by the step's LAST weight-update launch, on the CUs its tiles leave free
  // (tnet_affine_update_bias_gather) -- in stream order, so no cross-stream wait, and one launch less per
  // step.  Where the library does not take it (shapes, data parallelism, cross-validation), the gather is
  // launched right after the step.
  static const bool tail = !(getenv("TNET_GATHER_TAIL") && getenv("TNET_GATHER_TAIL")[0] == '0');
  TailGatherGuard guard(*mNet, cs);
  if (!mAhead && tail && mCache.HasBunchAhead()) {
    CuMatrix<BaseFloat>& nf = mFeatsB[mCur ^ 1];
    CuVector<int>& nl = mLabelsB[mCur ^ 1];
    nf.Init(mCache.Bunchsize(), mFeatsB[mCur].Cols());
    nl.Init(mCache.Bunchsize());
    // from here the cache has moved past that bunch: mAhead stays true and the guard delivers the bunch into
    // the other buffer whatever happens below (a throwing TrainBunch must not skip a bunch)
    // (data parallel: the network launches it right behind its last gradient GEMM, beside the exchange)
    guard.Arm(mCache.AheadGather(nf, nl), !mOpt.crossval);
    mAhead = true;
  }
  mNet->TrainBunch(mFeatsB[mCur], mLabelsB[mCur], *mObj, !mOpt.crossval, mOpt.crossval ? nullptr : mExchange);
  guard.Finish();
  if (mOpt.trace & 2) std::cout << "." << std::flush;
  mSteps++;
}

bool CuTrainer::DrainCache(bool final) {
  if (mOpt.randomize) mCache.Randomize();
  mTrainedSinceFill = true;
  if (DataParallel()) return DpRound((long)(mCache.IntakePos() / mCache.Bunchsize()), final);
  while (mAhead || !mCache.Empty()) Step();
  return true;
}

bool CuTrainer::DpRound(long n, bool final) {
  const DpRoundPlan plan = DpPlanRound(*mExchange, n, final);
  const size_t B = mCache.Bunchsize();
  for (long j = 0; j < plan.steps; j++) {
    mExchange->SetStepRows((size_t)plan.ranks_at_step[j] * B);
    if (j < n) {
      Step();
    } else {
      mNet->TrainEmpty(*mExchange);
      mEmptySteps++;
    }
  }
  mExchange->SetStepRows(0);
  return plan.all_final;
}

void CuTrainer::SetTransform(CuNetwork* transform, size_t start_ext, size_t end_ext) {
  mTransform = transform;
  mStartExt = transform ? start_ext : 0;
  mEndExt = transform ? end_ext : 0;
}

void CuTrainer::AddUtterance(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels) {
  CheckLabels(labels, rows, mNet->GetNOutputs(), "CuTrainer::AddUtterance");
  if (mTransform && rows > 0) {
    // frame extension on the host (the reader's job in the reference), one upload, the transform
    // network on the device, trim, then the cache takes the device rows
    const size_t R = rows + mStartExt + mEndExt;
    mExtHost.resize(R * cols);
    for (size_t r = 0; r < R; r++) {
      const size_t src = r < mStartExt ? 0 : (r - mStartExt >= rows ? rows - 1 : r - mStartExt);
      std::memcpy(&mExtHost[r * cols], feats + src * ld, cols * sizeof(float));
    }
    TransformAndAdd(mExtHost.data(), R, cols, cols, labels, rows);
    return;
  }
  if (cols != mNet->GetNInputs()) {
    std::ostringstream os;
    os << "CuTrainer::AddUtterance: feature dim " << cols << " != network input dim " << mNet->GetNInputs();
    Error(os.str());
  }
  if (rows == 0) return;
  mCache.AddDataHost(feats, rows, cols, ld, labels);
  mTrainedSinceFill = false;
  if (mCache.Full()) DrainCache(false);
}

void CuTrainer::TransformAndAdd(const float* ext, size_t rows_ext, size_t cols, size_t ld, const int* labels,
                                size_t rows) {
  mRaw.CopyFromHost(ext, rows_ext, cols, ld);
  mTransform->Propagate(mRaw, mTransformed);
  if (mTransformed.Cols() != mNet->GetNInputs()) {
    std::ostringstream os;
    os << "CuTrainer::AddUtterance: transformed feature dim " << mTransformed.Cols() << " != network input dim "
       << mNet->GetNInputs();
    Error(os.str());
  }
  mTrimmed.Init(rows, mTransformed.Cols());
  mTrimmed.CopyRows(rows, mStartExt, mTransformed, 0);
  mUttLabels.CopyFromHost(labels, rows);
  mCache.AddDataLabels(mTrimmed, mUttLabels);
  mTrainedSinceFill = false;
  if (mCache.Full()) DrainCache(false);
}

void CuTrainer::AddUtteranceExtended(const float* feats, size_t rows_ext, size_t cols, size_t ld, const int* labels,
                                     size_t start_ext, size_t end_ext) {
  if (rows_ext < start_ext + end_ext + 1) {
    std::ostringstream os;
    os << "CuTrainer::AddUtteranceExtended: " << rows_ext << " rows cannot carry " << start_ext << " + " << end_ext
       << " context rows";
    Error(os.str());
  }
  const size_t rows = rows_ext - start_ext - end_ext;
  if (!mTransform) {  // TNetCu.cc:390-393 trims the context whatever the (empty) transform
    AddUtterance(feats + start_ext * ld, rows, cols, ld, labels);
    return;
  }
  if (start_ext != mStartExt || end_ext != mEndExt) {
    std::ostringstream os;
    os << "CuTrainer::AddUtteranceExtended: features carry " << start_ext << "/" << end_ext
       << " context rows, the transform expects " << mStartExt << "/" << mEndExt;
    Error(os.str());
  }
  CheckLabels(labels, rows, mNet->GetNOutputs(), "CuTrainer::AddUtteranceExtended");
  TransformAndAdd(feats, rows_ext, cols, ld, labels, rows);
}

void CuTrainer::Finish() {
  // TNetCu.cc:376-441: after EndOfList the (partial) cache filled so far is drained once;
  // a leftover still pending after a full cache was drained is dropped.
  bool all_final = true;
  if (!mTrainedSinceFill && mCache.IntakePos() > 0) all_final = DrainCache(true);
  else if (DataParallel()) all_final = DpRound(0, true);
  // data-parallel: keep joining the other ranks' drains (zero gradients) until all are done
  while (!all_final) all_final = DpRound(0, true);
}

size_t CuTrainer::Prefill(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels) {
  if (mCache.Full()) return 0;
  const size_t space = mOpt.cachesize - mCache.IntakePos();
  const size_t take = rows < space ? rows : space;
  CheckLabels(labels, take, mNet->GetNOutputs(), "CuTrainer::Prefill");
  mCache.AddDataHost(feats, take, cols, ld, labels);
  if (mCache.Full() && mOpt.randomize) mCache.Randomize();
  return take;
}

void CuTrainer::Replay(long n) {
  for (long i = 0; i < n; i++) {
    if (!mAhead && mCache.Empty()) {
      mCache.Rewind();
      if (mOpt.randomize) mCache.Randomize();
    }
    Step();
  }
}

// ======================================================================================
// data-parallel step plan
// ======================================================================================
DpRoundPlan DpPlanRound(GradExchange& ex, long n, bool final) {
  const int world = ex.WorldSize(), rank = ex.Rank();
  if (n < 0) Error("DpPlanRound: negative bunch count");
  std::vector<double> info(2 * (size_t)world, 0.0);  // [n_r, final_r] per rank, summed = gathered
  info[2 * rank] = (double)n;
  info[2 * rank + 1] = final ? 1.0 : 0.0;
  ex.AllReduceHost(info.data(), (int)info.size());
  DpRoundPlan plan;
  for (int r = 0; r < world; r++) {
    plan.steps = std::max(plan.steps, (long)info[2 * r]);
    plan.all_final = plan.all_final && info[2 * r + 1] != 0.0;
  }
  plan.ranks_at_step.assign((size_t)plan.steps, 0);
  for (int r = 0; r < world; r++)
    for (long j = 0; j < (long)info[2 * r]; j++) plan.ranks_at_step[(size_t)j]++;
  return plan;
}

// ======================================================================================
// host-transport exchange
// ======================================================================================
// TNET_DP_SHARD=1: reduce-scatter + sharded apply + all-gather instead of the all-reduce.  Off by
// default on every transport until a multi-rank RCCL run has shown the sharded parameters equal the
// all-reduce path's (the protocol is tested over the host transport only).  Under sharding a rank's
// momentum buffers are valid only on its own shard (+ the tail): a later purely local update (no
// communicator) would let the replicas drift apart.
static bool shard_env() {
  const char* e = getenv("TNET_DP_SHARD");
  return e && e[0] == '1';
}

// every rank must run the same exchange form: one rank issuing reduce-scatter / all-gather while
// another issues all-reduce hangs or corrupts the collectives
static void check_same_shard_mode(GradExchange& ex, bool shard, int world) {
  double v[2] = {shard ? 1.0 : 0.0, 1.0};
  ex.AllReduceHost(v, 2);
  if (v[1] != (double)world) Error("GradExchange: rank count mismatch at communicator creation");
  if (v[0] != 0.0 && v[0] != (double)world)
    Error("GradExchange: ranks disagree on TNET_DP_SHARD (sharded apply on some ranks only)");
}

HostExchange::HostExchange(int rank, int world, HostAllReduceFn fn, void* user)
    : mRank(rank), mWorld(world), mShard(shard_env()),
      mInline(getenv("TNET_DP_HOST_INLINE") && getenv("TNET_DP_HOST_INLINE")[0] == '1'), mFn(fn), mUser(user) {
  check_same_shard_mode(*this, mShard, mWorld);
}

void* HostExchange::ApplyStream(int i) {
  (void)i;
  return mInline ? (void*)CuDevice::Instantiate().Stream() : nullptr;
}

int HostExchange::ApplyRanges(long n, long* lo, long* hi) const {
  return mShard ? ShardRanges(n, mRank, mWorld, lo, hi) : FullRange(n, lo, hi);
}

void HostExchange::GatherParams(CuUpdatableComponent& comp, int i, void* stream) {
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  (void)i;
  if (!mShard) return;
  CuDevice& dev = CuDevice::Instantiate();
  TNET_HIP_CALL(hipStreamSynchronize(stream ? (hipStream_t)stream : dev.Stream()));
  for (auto& b : comp.GradientBlocks()) {
    mStage.resize((size_t)b.n);
    TNET_HIP_CALL(hipMemcpy(mStage.data(), b.param, (size_t)b.n * sizeof(float), hipMemcpyDeviceToHost));
    const long c = ShardChunk(b.n, mWorld), main = c * mWorld;
    for (long k = 0; k < b.n; ++k) {
      const bool mine = k < main ? (k / c) == mRank : mRank == 0;
      if (!mine) mStage[(size_t)k] = 0.f;
    }
    if (mFn(mUser, mStage.data(), b.n, 0) != 0) Error("HostExchange: all-reduce callback failed");
    TNET_HIP_CALL(hipMemcpy(b.param, mStage.data(), (size_t)b.n * sizeof(float), hipMemcpyHostToDevice));
  }
}

// the device copies of the k-th submitted block (grown when a block is larger than the buffers it has)
void GradExchange::ReserveCapture(size_t k, long n) {
  while (mDevCap.size() <= k) mDevCap.emplace_back();
  DeviceCapture& c = mDevCap[k];
  if (c.cap >= n) return;
  if (c.local) TNET_HIP_CALL(hipFree(c.local));
  if (c.reduced) TNET_HIP_CALL(hipFree(c.reduced));
  c.local = c.reduced = nullptr;
  TNET_HIP_CALL(hipMalloc(&c.local, (size_t)n * sizeof(float)));
  TNET_HIP_CALL(hipMalloc(&c.reduced, (size_t)n * sizeof(float)));
  c.cap = n;
}

void GradExchange::ArmCapture(bool on) {
  mCaptureArmed = on;
  if (on) {
    mNumCaptured = 0;
    mCapturePending = false;
    mCaptured.clear();
    // the copies are allocated HERE, before the armed step, for the blocks the unarmed steps submitted (the same
    // blocks in the same order every step): the armed step itself then makes no allocation
    for (size_t k = 0; k < mSeen.size(); ++k) ReserveCapture(k, mSeen[k].second);
  }
}

size_t GradExchange::CaptureLocal(CuUpdatableComponent& comp, void* stream) {
  const size_t first = mNumCaptured;
  if (!mCaptureArmed) {
    // unarmed: the blocks of the latest step in submission order (host only, a few entries): a step starts again
    // when its first block recurs; a block out of the recorded order (another network on this exchange) cuts the
    // record there, so it never holds more than one step's blocks
    for (auto& b : comp.GradientBlocks()) {
      if (mSeenPos < mSeen.size() && mSeen[mSeenPos].first == b.param) {
        mSeen[mSeenPos].second = std::max(mSeen[mSeenPos].second, b.n);
      } else if (!mSeen.empty() && mSeen[0].first == b.param) {
        mSeenPos = 0;
        mSeen[0].second = std::max(mSeen[0].second, b.n);
      } else {
        mSeen.resize(mSeenPos);
        mSeen.emplace_back(b.param, b.n);
      }
      ++mSeenPos;
    }
    return first;
  }
  for (auto& b : comp.GradientBlocks()) {
    ReserveCapture(mNumCaptured, b.n);  // (allocates only for a block no unarmed step submitted)
    DeviceCapture& c = mDevCap[mNumCaptured++];
    c.n = b.n;
    c.nr = ApplyRanges(b.n, c.lo, c.hi);
    TNET_HIP_CALL(hipMemcpyAsync(c.local, b.grad, (size_t)b.n * sizeof(float), hipMemcpyDeviceToDevice,
                                 (hipStream_t)stream));
  }
  mCapturePending = true;
  return first;
}

void GradExchange::CaptureReduced(CuUpdatableComponent& comp, void* stream, size_t first) {
  if (!mCaptureArmed) return;
  size_t k = first;
  for (auto& b : comp.GradientBlocks()) {
    if (k >= mNumCaptured || mDevCap[k].n != b.n) Error("GradExchange: capture out of step with the submitted blocks");
    TNET_HIP_CALL(hipMemcpyAsync(mDevCap[k++].reduced, b.grad, (size_t)b.n * sizeof(float), hipMemcpyDeviceToDevice,
                                 (hipStream_t)stream));
  }
}

const std::vector<GradExchange::CapturedBlock>& GradExchange::Captured() {
  if (!mCapturePending) return mCaptured;
  TNET_HIP_CALL(hipDeviceSynchronize());  // after the armed step: every copy on every stream has landed
  mCaptured.assign(mNumCaptured, CapturedBlock{});
  std::vector<float> all;
  for (size_t i = 0; i < mNumCaptured; ++i) {
    const DeviceCapture& d = mDevCap[i];
    CapturedBlock& c = mCaptured[i];
    c.local.resize((size_t)d.n);
    all.resize((size_t)d.n);
    TNET_HIP_CALL(hipMemcpy(c.local.data(), d.local, (size_t)d.n * sizeof(float), hipMemcpyDeviceToHost));
    TNET_HIP_CALL(hipMemcpy(all.data(), d.reduced, (size_t)d.n * sizeof(float), hipMemcpyDeviceToHost));
    c.reduced.assign((size_t)d.n, std::numeric_limits<float>::quiet_NaN());
    for (int r = 0; r < d.nr; r++)
      std::copy(all.begin() + d.lo[r], all.begin() + d.hi[r], c.reduced.begin() + d.lo[r]);
  }
  mCapturePending = false;
  return mCaptured;
}

GradExchange::~GradExchange() {
  for (auto& c : mDevCap) {
    if (c.local) (void)hipFree(c.local);
    if (c.reduced) (void)hipFree(c.reduced);
  }
}

void HostExchange::Submit(CuUpdatableComponent& comp) {
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  CuDevice& dev = CuDevice::Instantiate();
  TNET_HIP_CALL(hipStreamSynchronize(dev.Stream()));
  const size_t first = CaptureLocal(comp, dev.Stream());
  for (auto& b : comp.GradientBlocks()) AllReduceDevice(b.grad, (size_t)b.n);
  CaptureReduced(comp, dev.Stream(), first);
}

bool HostExchange::SubmitInline(CuUpdatableComponent* const* comps, int n) {
  if (mShard || n <= 0) return false;
  for (int i = 0; i < n; ++i) Submit(*comps[i]);
  return true;
}

void HostExchange::AllReduceDevice(float* buf, size_t n) {
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  CuDevice& dev = CuDevice::Instantiate();
  mStage.resize(n);
  TNET_HIP_CALL(hipMemcpyAsync(mStage.data(), buf, n * sizeof(float), hipMemcpyDeviceToHost, dev.Stream()));
  TNET_HIP_CALL(hipStreamSynchronize(dev.Stream()));
  if (mFn(mUser, mStage.data(), (long)n, 0) != 0) Error("HostExchange: all-reduce callback failed");
  TNET_HIP_CALL(hipMemcpyAsync(buf, mStage.data(), n * sizeof(float), hipMemcpyHostToDevice, dev.Stream()));
  TNET_HIP_CALL(hipStreamSynchronize(dev.Stream()));
}

void HostExchange::AllReduceHost(double* v, int n) {
  if (n <= 0) return;
  if (mFn(mUser, v, (long)n, 1) != 0) Error("HostExchange: all-reduce callback failed");
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
  std::vector<hipEvent_t> events;     // compute stream -> comm stream (gradient ready), per submit
  std::vector<hipEvent_t> ar_done;    // comm stream -> compute stream (reduction done), per submit
  size_t next_event = 0;
  hipEvent_t done = nullptr;
  // applies of reduced layers: their own stream, so the comm stream only carries the reductions
  hipStream_t apply_stream = nullptr;
  hipEvent_t apply_done = nullptr;
  bool applied = false;
  std::vector<hipEvent_t> gather_ev;  // apply stream -> comm stream (a layer's shard applied), per submit
  double* dscratch = nullptr;
  // the comm stream's work in enqueue order (1, 2, ... per Submit / GatherParams), the position each
  // submission's ar_done marks, and how far the compute / apply stream has already waited: WaitAll skips its
  // own comm-stream wait when a stream it joins has covered everything (each wait is a barrier packet on the
  // compute queue, ~5.5 us even when satisfied: profiles/r04_dp_event_fence_ab.json)
  unsigned long comm_seq = 0, compute_covered = 0, apply_covered = 0;
  std::vector<unsigned long> ar_seq;
};

// RCCL channels and the CUs reserved for them.  RCCL runs one workgroup per channel (512 threads,
// 37.6 KB LDS, 248-256 VGPRs, resident for the whole collective: tools/cohab_probe.hip), and a GEMM
// grid of exactly one tile round per CU loses a whole second round beside them (1.8x,
// profiles/r02_rccl_cohab_probe.txt).  So the channel count is capped (NCCL_MAX_NCHANNELS, when the
// user has not set it: TNET_DP_RCCL_CHANNELS, default 16) and while this rank's reductions are in
// flight the GEMMs run stream-K over CUs - R workgroups, R = the cap (TNET_DP_RESERVE_CUS overrides;
// 0: off).  Single-rank communicators launch no channel kernels: no reservation unless asked for.
// the cap, set before RCCL reads its environment (UniqueId on rank 0, the communicator on every rank)
static int rccl_channels() {
  const char* mx = getenv("NCCL_MAX_NCHANNELS");
  if (mx) return atoi(mx);
  const char* ch = getenv("TNET_DP_RCCL_CHANNELS");
  const int channels = ch ? atoi(ch) : 16;
  if (channels > 0) setenv("NCCL_MAX_NCHANNELS", std::to_string(channels).c_str(), 0);
  return channels;
}
// The exchange's stream-ordering events (compute -> comm -> apply -> compute): every consumer is a stream of
// this device (RCCL's kernels, the applies, the next GEMMs), and a kernel's completion already releases its
// stores at device scope, so the events are recorded without HIP's default system-scope fence (L2 write-back
// + invalidate at every record: the one-rank DP step showed 6-26 us compute-stream bubbles at each of the
// step's exchange points, profiles/r04_dp_event_fence_ab.json).  TNET_DP_EVENT_FENCE=1: the default fence.
static unsigned exchange_event_flags() {
  static const bool fence = getenv("TNET_DP_EVENT_FENCE") && getenv("TNET_DP_EVENT_FENCE")[0] == '1';
  return hipEventDisableTiming | (fence ? 0u : (unsigned)hipEventDisableSystemFence);
}
static int rccl_reserve(int world) {
  const int channels = rccl_channels();
  const char* rv = getenv("TNET_DP_RESERVE_CUS");  // explicit: also at world 1 (tests)
  if (rv) return atoi(rv) > 0 ? atoi(rv) : 0;
  return world > 1 && channels > 0 ? channels : 0;
}

void RcclExchange::UniqueId(char out[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  (void)rccl_channels();
  NCCL_CALL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, 128);
}

RcclExchange::RcclExchange(int rank, int world, const char id[128])
    : mImpl(new Impl), mRank(rank), mWorld(world), mShard(shard_env()), mReserve(rccl_reserve(world)) {
  CuDevice& dev = CuDevice::Instantiate();
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  NCCL_CALL(ncclCommInitRank(&mImpl->comm, world, uid, rank));
  TNET_HIP_CALL(hipStreamCreateWithFlags(&mImpl->comm_stream, hipStreamNonBlocking));
  TNET_HIP_CALL(hipStreamCreateWithFlags(&mImpl->apply_stream, hipStreamNonBlocking));
  TNET_HIP_CALL(hipEventCreateWithFlags(&mImpl->done, exchange_event_flags()));
  TNET_HIP_CALL(hipEventCreateWithFlags(&mImpl->apply_done, exchange_event_flags()));
  TNET_HIP_CALL(hipMalloc(&mImpl->dscratch, 4096));
  (void)dev;
  check_same_shard_mode(*this, mShard, mWorld);
}

RcclExchange::~RcclExchange() {
  if (!mImpl) return;
  (void)hipStreamSynchronize(mImpl->comm_stream);
  if (mImpl->apply_stream) (void)hipStreamSynchronize(mImpl->apply_stream);
  for (auto e : mImpl->events) (void)hipEventDestroy(e);
  for (auto e : mImpl->ar_done) (void)hipEventDestroy(e);
  for (auto e : mImpl->gather_ev) (void)hipEventDestroy(e);
  if (mImpl->done) (void)hipEventDestroy(mImpl->done);
  if (mImpl->apply_done) (void)hipEventDestroy(mImpl->apply_done);
  if (mImpl->apply_stream) (void)hipStreamDestroy(mImpl->apply_stream);
  if (mImpl->dscratch) (void)hipFree(mImpl->dscratch);
  if (mImpl->comm) (void)ncclCommDestroy(mImpl->comm);
  if (mImpl->comm_stream) (void)hipStreamDestroy(mImpl->comm_stream);
}

void RcclExchange::Submit(CuUpdatableComponent& comp) {
  CuDevice& dev = CuDevice::Instantiate();
  if (mImpl->next_event >= mImpl->events.size()) {
    hipEvent_t e, d;
    TNET_HIP_CALL(hipEventCreateWithFlags(&e, exchange_event_flags()));
    TNET_HIP_CALL(hipEventCreateWithFlags(&d, exchange_event_flags()));
    mImpl->events.push_back(e);
    mImpl->ar_done.push_back(d);
    mImpl->ar_seq.push_back(0);
  }
  const size_t idx = mImpl->next_event++;
  if (idx == 0 && mReserve > 0) TNET_SAFE_CALL(tnet_gemm_reserve(mReserve));
  hipEvent_t ev = mImpl->events[idx];
  // the gradient kernels were enqueued on the compute stream: order the reduction after them
  TNET_HIP_CALL(hipEventRecord(ev, dev.Stream()));
  TNET_HIP_CALL(hipStreamWaitEvent(mImpl->comm_stream, ev, 0));
  const size_t first = CaptureLocal(comp, mImpl->comm_stream);
  std::vector<CuParamBlock> blocks = comp.GradientBlocks();
  NCCL_CALL(ncclGroupStart());
  for (auto& b : blocks) {
    if (!mShard) {
      NCCL_CALL(ncclAllReduce(b.grad, b.grad, (size_t)b.n, ncclFloat, ncclSum, mImpl->comm, mImpl->comm_stream));
      continue;
    }
    // in place: this rank's reduced shard lands at grad + rank * c; the tail is reduced whole
    const long c = ShardChunk(b.n, mWorld), main = c * mWorld;
    if (c > 0)
      NCCL_CALL(ncclReduceScatter(b.grad, b.grad + (long)mRank * c, (size_t)c, ncclFloat, ncclSum, mImpl->comm,
                                  mImpl->comm_stream));
    if (main < b.n)
      NCCL_CALL(ncclAllReduce(b.grad + main, b.grad + main, (size_t)(b.n - main), ncclFloat, ncclSum, mImpl->comm,
                              mImpl->comm_stream));
  }
  NCCL_CALL(ncclGroupEnd());
  // armed: the reduced copy sits in the comm stream's order before ar_done, so nothing that waits for this
  // reduction (the apply, the next step's gradient GEMM writing G again) can run before it has read G
  CaptureReduced(comp, mImpl->comm_stream, first);
  TNET_HIP_CALL(hipEventRecord(mImpl->ar_done[idx], mImpl->comm_stream));
  mImpl->ar_seq[idx] = ++mImpl->comm_seq;
}

// The step's whole reduction on the compute stream (GradExchange::SubmitInline): all-reduce only (the sharded form
// keeps its per-layer reduce-scatter / apply / all-gather order on the comm stream), and only as the step's sole
// submission -- so every collective of a step is on ONE stream (RCCL serialises a communicator's operations across
// streams itself, but the exchange never relies on it: the synchronous AllReduceHost / AllReduceDevice drain both
// streams around their comm-stream call).  No CU reservation: no GEMM runs beside these collectives.
// TNET_DP_INLINE=0: the per-layer Submit path (A/B).
bool RcclExchange::SubmitInline(CuUpdatableComponent* const* comps, int n) {
  static const bool off = getenv("TNET_DP_INLINE") && getenv("TNET_DP_INLINE")[0] == '0';
  if (off || mShard || n <= 0 || mImpl->next_event != 0) return false;
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  const hipStream_t cs = CuDevice::Instantiate().Stream();
  std::vector<size_t> first((size_t)n);
  for (int i = 0; i < n; ++i) first[(size_t)i] = CaptureLocal(*comps[i], cs);
  NCCL_CALL(ncclGroupStart());
  for (int i = 0; i < n; ++i)
    for (auto& b : comps[i]->GradientBlocks())
      NCCL_CALL(ncclAllReduce(b.grad, b.grad, (size_t)b.n, ncclFloat, ncclSum, mImpl->comm, cs));
  NCCL_CALL(ncclGroupEnd());
  for (int i = 0; i < n; ++i) CaptureReduced(*comps[i], cs, first[(size_t)i]);
  return true;
}

int RcclExchange::TransportRanks() const {
  int n = 0;
  NCCL_CALL(ncclCommCount(mImpl->comm, &n));
  return n;
}

int RcclExchange::ApplyRanges(long n, long* lo, long* hi) const {
  return mShard ? ShardRanges(n, mRank, mWorld, lo, hi) : FullRange(n, lo, hi);
}

void RcclExchange::GatherParams(CuUpdatableComponent& comp, int i, void* stream) {
  if (!mShard) return;
  if (i < 0 || (size_t)i >= mImpl->next_event) Error("RcclExchange::GatherParams: no such reduction");
  // the comm stream waits for this layer's applies (their stream), then all-gathers the shards in
  // place: the next collectives queue behind it, the compute stream joins at WaitAll
  while (mImpl->gather_ev.size() <= (size_t)i) {
    hipEvent_t e;
    TNET_HIP_CALL(hipEventCreateWithFlags(&e, exchange_event_flags()));
    mImpl->gather_ev.push_back(e);
  }
  if ((hipStream_t)stream != mImpl->comm_stream) {  // applied on the comm stream: already in its order
    hipEvent_t ev = mImpl->gather_ev[(size_t)i];
    TNET_HIP_CALL(hipEventRecord(ev, stream ? (hipStream_t)stream : CuDevice::Instantiate().Stream()));
    TNET_HIP_CALL(hipStreamWaitEvent(mImpl->comm_stream, ev, 0));
  }
  NCCL_CALL(ncclGroupStart());
  for (auto& b : comp.GradientBlocks()) {
    const long c = ShardChunk(b.n, mWorld);
    if (c > 0)
      NCCL_CALL(ncclAllGather(b.param + (long)mRank * c, b.param, (size_t)c, ncclFloat, mImpl->comm,
                              mImpl->comm_stream));
  }
  NCCL_CALL(ncclGroupEnd());
  ++mImpl->comm_seq;
}

void RcclExchange::WaitFor(int i) {
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  if (i < 0 || (size_t)i >= mImpl->next_event) Error("RcclExchange::WaitFor: no such reduction");
  TNET_HIP_CALL(hipStreamWaitEvent(CuDevice::Instantiate().Stream(), mImpl->ar_done[(size_t)i], 0));
  mImpl->compute_covered = std::max(mImpl->compute_covered, mImpl->ar_seq[(size_t)i]);
}

// A layer's apply goes on the comm stream right behind its own reduction (no hop: stream order), beside the
// backward GEMMs still on the compute stream; the next reduction queues behind it, which costs nothing -- the next
// layer's gradient takes a whole backward GEMM to exist.  The apply counts as comm-stream work, so a WaitFor on a
// later reduction covers it and WaitAll joins only what no wait covered (the round-4 form, a separate apply stream
// with a hop in per layer and a join out per step: TNET_DP_APPLY_COMM=0).
void* RcclExchange::ApplyStream(int i) {
  static const bool off = getenv("TNET_DP_APPLY_STREAM") && getenv("TNET_DP_APPLY_STREAM")[0] == '0';
  static const bool on_comm = !(getenv("TNET_DP_APPLY_COMM") && getenv("TNET_DP_APPLY_COMM")[0] == '0');
  if (off) return nullptr;  // A/B: the applies on the compute stream after WaitFor (round-1 form)
  if (i < 0 || (size_t)i >= mImpl->next_event) Error("RcclExchange::ApplyStream: no such reduction");
  if (on_comm) {
    ++mImpl->comm_seq;  // the apply the caller enqueues next
    return (void*)mImpl->comm_stream;
  }
  TNET_HIP_CALL(hipStreamWaitEvent(mImpl->apply_stream, mImpl->ar_done[(size_t)i], 0));
  mImpl->apply_covered = std::max(mImpl->apply_covered, mImpl->ar_seq[(size_t)i]);
  mImpl->applied = true;
  return (void*)mImpl->apply_stream;
}

void RcclExchange::WaitAll() {
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  CuDevice& dev = CuDevice::Instantiate();
  // the comm stream's work is already behind the compute stream when it (or the apply stream it joins below)
  // waited for the comm stream's last enqueued operation (TNET_DP_WAITALL_COMM=1: wait anyway, A/B)
  static const bool always = getenv("TNET_DP_WAITALL_COMM") && getenv("TNET_DP_WAITALL_COMM")[0] == '1';
  const bool covered = mImpl->compute_covered == mImpl->comm_seq ||
                       (mImpl->applied && mImpl->apply_covered == mImpl->comm_seq);
  if (always || !covered) {
    TNET_HIP_CALL(hipEventRecord(mImpl->done, mImpl->comm_stream));
    TNET_HIP_CALL(hipStreamWaitEvent(dev.Stream(), mImpl->done, 0));
  }
  if (mImpl->applied) {
    TNET_HIP_CALL(hipEventRecord(mImpl->apply_done, mImpl->apply_stream));
    TNET_HIP_CALL(hipStreamWaitEvent(dev.Stream(), mImpl->apply_done, 0));
    mImpl->applied = false;
  }
  mImpl->comm_seq = mImpl->compute_covered = mImpl->apply_covered = 0;
  mImpl->next_event = 0;
  if (mReserve > 0) TNET_SAFE_CALL(tnet_gemm_reserve(0));
  DisarmCapture();
}

void RcclExchange::AllReduceHost(double* v, int n) {
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
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
  CuDevice::Instantiate().KTCloseRun();  // no roofline timing run spans an exchange step
  CuDevice& dev = CuDevice::Instantiate();
  TNET_HIP_CALL(hipStreamSynchronize(dev.Stream()));
  NCCL_CALL(ncclAllReduce(buf, buf, n, ncclFloat, ncclSum, mImpl->comm, mImpl->comm_stream));
  TNET_HIP_CALL(hipStreamSynchronize(mImpl->comm_stream));
}

}  // namespace TNet
