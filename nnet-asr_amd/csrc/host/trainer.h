// trainer.h -- the TNetCu SGD loop (src/TNetCu.cc:375-442) as a library object, plus the RCCL
// data-parallel gradient exchange.
//
// Loop semantics kept from the reference driver: utterances are appended to the cache in scp
// order; when the cache is full it is shuffled (if RANDOMIZE) and drained bunch by bunch, each
// bunch = Propagate -> objective -> Backpropagate(+Update) (or forward+objective only for
// cross-validation); after the last utterance the partially filled cache is drained the same
// way and a pending leftover is dropped, exactly as TNetCu's outer while(!EndOfList) does.
// Cache size is rounded down to a multiple of the bunch size (TNetCu.cc:362).
#pragma once

#include <memory>

#include "cucache.h"
#include "cunetwork.h"
#include "gradexchange.h"

namespace TNet {

struct TrainerOptions {
  size_t bunchsize = 256;     // --BUNCHSIZE (TNetCu.cc:225)
  size_t cachesize = 12800;   // --CACHESIZE (TNetCu.cc:226)
  long seed = 0;              // --SEED (0 = time seeded, TNetCu.cc:330-338)
  bool randomize = true;      // --RANDOMIZE
  bool crossval = false;      // --CROSSVALIDATE / -c
  int trace = 0;              // --TRACE
};

class CuTrainer {
 public:
  CuTrainer(CuNetwork* net, CuObjectiveFunction* obj, const TrainerOptions& opt);
  ~CuTrainer();

  /// Data-parallel mode: gradients are summed over ranks every step (ranks must take the same
  /// number of steps).
  void SetExchange(GradExchange* ex) { mExchange = ex; }

  /// --FEATURETRANSFORM + --STARTFRMEXT/--ENDFRMEXT (TNetCu.cc:274-278, 384-393): every utterance
  /// is extended by repeating its first/last frame (the KaldiLib reader, Features.cc:776-850),
  /// pushed through `transform` on the device and trimmed before it enters the cache.  The
  /// transform network is borrowed (not owned); nullptr switches it off.
  void SetTransform(CuNetwork* transform, size_t start_ext, size_t end_ext);

  /// Append one utterance (host memory): features [rows x cols] with leading dim ld, class ids.
  void AddUtterance(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels);
  /// Append one utterance as the reference's FeatureRepository delivers it (TNetCu.cc:385-416):
  /// `rows_ext` rows that already carry `start_ext` / `end_ext` context rows (edge replication, or
  /// real neighbouring frames of a [s,e] range), labels for the rows_ext - start_ext - end_ext frames
  /// between.  With a transform, the extension must be the transform's; without, the context rows
  /// are trimmed.
  void AddUtteranceExtended(const float* feats, size_t rows_ext, size_t cols, size_t ld, const int* labels,
                            size_t start_ext, size_t end_ext);
  /// End of the utterance list.
  void Finish();
  /// Steps (bunches) trained so far.
  long Steps() const { return mSteps; }
  /// Data-parallel steps this rank joined without a bunch of its own (zero gradient).
  long EmptySteps() const { return mEmptySteps; }
  /// Fill the cache from host utterances WITHOUT training (benchmark setup); returns the
  /// number of rows taken.  The cache is shuffled once filled.
  size_t Prefill(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels);
  /// Benchmark replay: run n more SGD steps over the resident cache contents, re-shuffling
  /// (same RNG stream) every time the cache is exhausted.  The cache must have been filled.
  void Replay(long n);
  CuCache& Cache() { return mCache; }
  Rng48& Rng() { return mRng; }

 private:
  /// Shuffle and train every bunch of the cache; in data-parallel mode one planned round
  /// (DpPlanRound).  Returns whether every rank has reached its final drain.
  bool DrainCache(bool final);
  bool DpRound(long n, bool final);
  /// extended host rows -> transform on the device -> trim -> cache
  void TransformAndAdd(const float* ext, size_t rows_ext, size_t cols, size_t ld, const int* labels, size_t rows);
  bool DataParallel() const { return mExchange && !mOpt.crossval && mExchange->WorldSize() > 1; }
  void Step();

  CuNetwork* mNet;
  CuObjectiveFunction* mObj;
  TrainerOptions mOpt;
  GradExchange* mExchange = nullptr;
  CuCache mCache;
  Rng48 mRng;
  // bunch buffers: the step trains buffer mCur while its last launch gathers the next shuffled bunch of the
  // fill into the other one (CuNetwork::SetTailGather)
  CuMatrix<BaseFloat> mFeatsB[2];
  CuVector<int> mLabelsB[2];
  int mCur = 0;
  bool mAhead = false;        // buffer mCur ^ 1 holds the next bunch (gathered ahead, in stream order)
  CuNetwork* mTransform = nullptr;
  size_t mStartExt = 0, mEndExt = 0;
  std::vector<float> mExtHost;
  CuMatrix<BaseFloat> mRaw, mTransformed, mTrimmed;
  CuVector<int> mUttLabels;
  long mSteps = 0;
  long mEmptySteps = 0;
  bool mTrainedSinceFill = false;
};

/// Host-transport exchange: gradients are staged to host memory and summed by a caller-supplied
/// all-reduce (e.g. torch.distributed gloo, MPI).  Synchronous and PCIe-bound: for multi-node
/// transports without RCCL and for exercising the data-parallel path with several processes on
/// one device in tests.  fn(user, buf, n, is_double) must sum buf over ranks in place, return 0.
typedef int (*HostAllReduceFn)(void* user, void* buf, long n, int is_double);
class HostExchange : public GradExchange {
 public:
  HostExchange(int rank, int world, HostAllReduceFn fn, void* user);
  int Rank() const override { return mRank; }
  int WorldSize() const override { return mWorld; }
  void Submit(CuUpdatableComponent& comp) override;
  /// Submit is synchronous: the whole step's reduction is simply every component's, in order (not under
  /// TNET_DP_SHARD, whose applies and gathers go per layer)
  bool SubmitInline(CuUpdatableComponent* const* comps, int n) override;
  void WaitAll() override { DisarmCapture(); }
  void AllReduceHost(double* v, int n) override;
  void AllReduceDevice(float* buf, size_t n);
  /// TNET_DP_SHARD=1: the sharded-apply protocol of RcclExchange emulated through the host
  /// all-reduce (full reduction; each rank applies its ranges; the parameter blocks are then summed
  /// with every element outside the rank's shard zeroed, rank 0 contributing the tails) -- a test
  /// of the shard split on one device, not a fast path
  int ApplyRanges(long n, long* lo, long* hi) const override;
  void GatherParams(CuUpdatableComponent& comp, int i, void* stream) override;
  /// TNET_DP_HOST_INLINE=1: hand out the compute stream as the apply stream (Submit is synchronous,
  /// so the layer's reduction is done), which puts CuNetwork on the per-layer reduce -> apply ->
  /// gather order RcclExchange takes -- tests of that collective order with several ranks
  void* ApplyStream(int i) override;

 private:
  int mRank, mWorld;
  bool mShard = false;
  bool mInline = false;
  HostAllReduceFn mFn;
  void* mUser;
  std::vector<float> mStage;
};

/// RCCL all-reduce over xGMI, one communicator per rank (one process per GPU).
class RcclExchange : public GradExchange {
 public:
  static void UniqueId(char out[128]);
  RcclExchange(int rank, int world, const char id[128]);
  ~RcclExchange();
  int Rank() const override { return mRank; }
  int WorldSize() const override { return mWorld; }
  void Submit(CuUpdatableComponent& comp) override;
  bool SubmitInline(CuUpdatableComponent* const* comps, int n) override;
  void WaitAll() override;
  void WaitFor(int i) override;
  void* ApplyStream(int i) override;
  void AllReduceHost(double* v, int n) override;
  /// all-reduce (sum) of a device float buffer on the communication stream, synchronous
  void AllReduceDevice(float* buf, size_t n);
  /// Sharded apply (TNET_DP_SHARD=1 on every rank; off by default): Submit
  /// reduce-scatters each gradient block (ShardRanges; the tail all-reduced), the rank applies its
  /// shard, GatherParams all-gathers the updated parameters in place on the communication stream --
  /// the apply's HBM traffic divided by the world size, the same bytes over xGMI as an all-reduce
  int ApplyRanges(long n, long* lo, long* hi) const override;
  void GatherParams(CuUpdatableComponent& comp, int i, void* stream) override;
  int TransportRanks() const override;

 private:
  struct Impl;
  std::unique_ptr<Impl> mImpl;
  int mRank, mWorld;
  bool mShard = false;
  // CUs the 2048^2-class GEMMs leave to RCCL's channel workgroups while collectives are in flight
  // (tnet_gemm_reserve: stream-K over CUs - R workgroups from the first Submit of a step to WaitAll)
  int mReserve = 0;
};

}  // namespace TNet
