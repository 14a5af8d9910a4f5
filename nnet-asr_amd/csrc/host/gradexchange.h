// gradexchange.h -- data-parallel gradient exchange interface used by CuNetwork::TrainBunch.
//
// The reference has no multi-GPU path; its CPU Platform sums per-thread
// gradients row-slice by row-slice into a shared accumulator (src/TNetLib/Platform.h:307-335,
// BiasedLinearity.cc:90-178).  On MI355X the same "sum of the ranks' gradients, then one identical
// update everywhere" is an RCCL all-reduce over xGMI, issued per layer as soon as that layer's
// gradient exists, on a communication stream, so it overlaps the backward GEMMs of the layers
// below (rccl_exchange.cpp).
#pragma once

#include <cstddef>
#include <functional>
#include <utility>
#include <vector>

namespace TNet {

class CuUpdatableComponent;

class GradExchange {
 public:
  virtual ~GradExchange();
  virtual int Rank() const = 0;
  virtual int WorldSize() const = 0;
  /// Called after comp.ComputeGradient() was enqueued on the compute stream: start reducing
  /// comp.GradientBlocks() asynchronously.
  virtual void Submit(CuUpdatableComponent& comp) = 0;
  /// Make the compute stream wait until every submitted reduction has finished.
  virtual void WaitAll() = 0;
  /// Make the compute stream wait for the i-th reduction submitted since the last WaitAll() (the
  /// apply of that layer can then overlap the reductions still running); default: WaitAll().
  virtual void WaitFor(int i) {
    (void)i;
    WaitAll();
  }
  /// Stream on which the apply (SGD update) of the i-th submitted layer may be enqueued so that it
  /// runs as soon as that layer's reduction is done, beside the backward GEMMs still running on the
  /// compute stream; WaitAll() then also joins the applies.  nullptr: apply on the compute stream
  /// after WaitFor(i) (host transports, whose Submit is synchronous).
  virtual void* ApplyStream(int i) {
    (void)i;
    return nullptr;
  }
  /// The step's WHOLE reduction in one go, when every trained layer's gradient already exists (no backward GEMM is
  /// left for the reductions to overlap -- a network whose last gradient launch computed all of them, e.g. MLP3's
  /// two-gradient + gather launch): the collectives go on the compute stream right behind the gradient kernels, as
  /// one group, with no stream hop in and none out, and the caller applies each component on the compute stream
  /// (ApplyGradient with no stream, then GatherParams(comp, -1, nullptr)).  Returns false when the transport does
  /// not take this form (then Submit each component).  Only before the step's first Submit.
  virtual bool SubmitInline(CuUpdatableComponent* const* comps, int n) {
    (void)comps;
    (void)n;
    return false;
  }
  /// Sum small host statistics over ranks (epoch-end MergeStats, step planning); blocking.
  virtual void AllReduceHost(double* v, int n) = 0;

  // ---- sharded apply (ZeRO-1 style: reduce-scatter, each rank updates its shard, all-gather)
  /// The element ranges [lo[k], hi[k]) of an n-element block this rank applies after the block's
  /// reduction; returns the range count (<= 2).  Default: the whole block.
  virtual int ApplyRanges(long n, long* lo, long* hi) const { return FullRange(n, lo, hi); }
  /// After submission i's applies were enqueued (on `stream`; nullptr = the compute stream): bring
  /// every rank's updated elements of comp's parameter blocks.  No-op without sharding.
  virtual void GatherParams(CuUpdatableComponent& comp, int i, void* stream) {
    (void)comp;
    (void)i;
    (void)stream;
  }
  static int FullRange(long n, long* lo, long* hi) {
    lo[0] = 0;
    hi[0] = n;
    return 1;
  }
  /// The shard split of an n-element block over `world` ranks: rank r owns [r c, (r + 1) c) with c
  /// a multiple of 4 elements (16-byte aligned shards), every rank also applies the tail [world c, n)
  /// (fewer than 4 world elements, all-reduced whole).  Returns c.
  static long ShardChunk(long n, int world) { return (n / (4L * world)) * 4L; }
  static int ShardRanges(long n, int rank, int world, long* lo, long* hi) {
    const long c = ShardChunk(n, world), main = c * world;
    int k = 0;
    if (c > 0) {
      lo[k] = rank * c;
      hi[k++] = rank * c + c;
    }
    if (main < n) {
      lo[k] = main;
      hi[k++] = n;
    }
    return k;
  }

  /// Frames of the global bunch (sum over ranks) for the GRADDIVFRM normalisation: the row
  /// count planned for this step (SetStepRows), else every rank is assumed to hold local_rows.
  size_t GlobalRows(size_t local_rows) const {
    return mStepRows ? mStepRows : local_rows * (size_t)WorldSize();
  }
  void SetStepRows(size_t rows) { mStepRows = rows; }

  // ---- reduction check (bench.py rccl_check): armed for one step, every submitted gradient block is copied on the
  // DEVICE right before its reduction (this rank's local gradient: a D2D copy enqueued on the stream the reduction
  // runs on, after its wait for the gradient kernels -- the exact bytes RCCL reads) and right after it (the reduced
  // values, on the same stream behind the collective).  No host synchronisation inside the step, so the armed step
  // runs the production schedule; the copies are read back when the caller asks for them (Captured(), after the
  // step), the reduced ones restricted to the ranges this rank applies (NaN elsewhere).
  struct CapturedBlock {
    std::vector<float> local, reduced;
  };
  void ArmCapture(bool on);
  /// the armed step's blocks in submission order (synchronises the device and reads the copies back once)
  const std::vector<CapturedBlock>& Captured();
  /// the communicator's rank count as the transport reports it (ncclCommCount for RCCL)
  virtual int TransportRanks() const { return WorldSize(); }

 protected:
  /// Submit's halves of the capture (no-ops unless armed; `stream` is the stream the reduction is enqueued on:
  /// CaptureLocal right after its wait for the gradient kernels, CaptureReduced right behind the collective)
  /// (CaptureLocal returns the index of comp's first captured block, which CaptureReduced takes)
  size_t CaptureLocal(CuUpdatableComponent& comp, void* stream);
  void CaptureReduced(CuUpdatableComponent& comp, void* stream, size_t first);
  void DisarmCapture() { mCaptureArmed = false; }
  bool mCaptureArmed = false;

 private:
  size_t mStepRows = 0;
  // one captured block: its device copies (local, reduced) and the ranges this rank applied
  struct DeviceCapture {
    float* local = nullptr;
    float* reduced = nullptr;
    long n = 0, cap = 0;
    long lo[2] = {0, 0}, hi[2] = {0, 0};
    int nr = 0;
  };
  std::vector<DeviceCapture> mDevCap;  // buffers kept across arms (allocated when arming, ReserveCapture)
  std::vector<std::pair<const float*, long>> mSeen;  // the latest unarmed step's blocks: parameter address, size
  size_t mSeenPos = 0;                                 // the next block's position in that step
  void ReserveCapture(size_t k, long n);
  size_t mNumCaptured = 0;
  bool mCapturePending = false;        // device copies not yet read back
  std::vector<CapturedBlock> mCaptured;
};

/// One round of the data-parallel step plan (see DpPlanRound).
struct DpRoundPlan {
  long steps = 0;                 // max over ranks of the bunches of this round
  std::vector<int> ranks_at_step; // [steps]: ranks that hold a bunch at step j
  bool all_final = true;          // every rank has reached the end of its utterance list
};

/// Ranks fill their caches from different utterance shards, so at a cache drain they may hold
/// different numbers of bunches (always at the last, partial drain; and a rank may run out of
/// utterances whole drains earlier than another).  Every rank calls this once per drain with
/// its bunch count and whether this is its final drain; all ranks get the same plan: the round
/// lasts max(n_r) steps, a rank past its own n_r contributes a zero gradient, and step j
/// normalises by the rows of the ranks_at_step[j] ranks that trained.  A rank that has finished
/// keeps joining rounds with n = 0 until all_final.  (The reference's Platform slices one
/// global bunch over threads instead and never sees unequal shards: Platform.h:206-236.)
DpRoundPlan DpPlanRound(GradExchange& ex, long n, bool final);

}  // namespace TNet
