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

  /// Append one utterance (host memory): features [rows x cols] with leading dim ld, class ids.
  void AddUtterance(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels);
  /// End of the utterance list.
  void Finish();
  /// Steps (bunches) trained so far.
  long Steps() const { return mSteps; }
  /// Fill the cache from host utterances WITHOUT training (benchmark setup); returns the
  /// number of rows taken.  The cache is shuffled once filled.
  size_t Prefill(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels);
  /// Benchmark replay: run n more SGD steps over the resident cache contents, re-shuffling
  /// (same RNG stream) every time the cache is exhausted.  The cache must have been filled.
  void Replay(long n);
  CuCache& Cache() { return mCache; }
  Rng48& Rng() { return mRng; }

 private:
  void DrainCache();
  void Step();

  CuNetwork* mNet;
  CuObjectiveFunction* mObj;
  TrainerOptions mOpt;
  GradExchange* mExchange = nullptr;
  CuCache mCache;
  Rng48 mRng;
  CuMatrix<BaseFloat> mFeats;
  CuVector<int> mLabels;
  long mSteps = 0;
  bool mTrainedSinceFill = false;
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
  void WaitAll() override;
  size_t GlobalRows(size_t local_rows) override { return local_rows * (size_t)mWorld; }
  void AllReduceHost(double* v, int n) override;
  /// all-reduce (sum) of a device float buffer on the communication stream, synchronous
  void AllReduceDevice(float* buf, size_t n);

 private:
  struct Impl;
  std::unique_ptr<Impl> mImpl;
  int mRank, mWorld;
};

}  // namespace TNet
