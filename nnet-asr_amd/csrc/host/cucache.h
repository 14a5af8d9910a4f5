// cucache.h -- GPU-resident feature/target cache (src/CuTNetLib/cuCache.h:12-70, .cc:22-200).
//
// Same state machine as the reference: EMPTY -> INTAKE -> FULL -> EXHAUST, leftover rows of the
// utterance that overflowed carried into the next fill (truncated to the cache size), shuffle of
// the intake rows with lrand48 + libstdc++ random_shuffle, consecutive bunches, tail < bunch
// discarded.
//
// MI355X changes:
//   * Randomize() only draws the permutation (host LCG, identical stream to srand48/lrand48) and
//     uploads it; GetBunch() gathers the bunch rows straight from the intake buffer (one
//     row-gather kernel) instead of materialising a shuffled copy of the whole cache -- same
//     rows, half the HBM traffic;
//   * one-hot targets are held as class ids (4 B/frame; a 4000-senone one-hot cache row is
//     16 KB); a dense-target mode keeps the reference's AddData(features, desired) API;
//   * the cache is double-buffered and a host intake (AddDataHost) copies on its own copy stream:
//     the next fill streams in over PCIe while the GPU still trains on the previous one (the
//     compute stream waits for the copies once, when the new fill starts being exhausted; the copy
//     stream waits, before writing a buffer, for the gathers of the fill that last used it).
//     Leftover buffers are allocated once at the cache size (no allocation between the streams).
#pragma once

#include <thread>

#include "cumatrix.h"
#include "rng48.h"

namespace TNet {

class CuCache {
  typedef enum { EMPTY, INTAKE, FULL, EXHAUST } State;

 public:
  CuCache();
  ~CuCache();

  /// Initialize the cache (cachesize must be divisible by bunchsize)
  void Init(size_t cachesize, size_t bunchsize);
  /// Random stream used by Randomize (defaults to the process stream seeded by SeedRandom)
  void SetRng(Rng48* rng) { mRng = rng; }

  /// Dense targets (reference API)
  void AddData(const CuMatrix<BaseFloat>& rFeatures, const CuMatrix<BaseFloat>& rDesired);
  /// Class-id targets (device features + device labels)
  void AddDataLabels(const CuMatrix<BaseFloat>& rFeatures, const CuVector<int>& rLabels);
  /// Host utterance straight into the cache rows (no intermediate device copy)
  void AddDataHost(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels);

  void Randomize();
  void GetBunch(CuMatrix<BaseFloat>& rFeatures, CuMatrix<BaseFloat>& rDesired);
  void GetBunchLabels(CuMatrix<BaseFloat>& rFeatures, CuVector<int>& rLabels);
  /// Another bunch of the shuffled class-id fill being exhausted follows the one just taken (it can be
  /// gathered ahead: AheadGather)
  bool HasBunchAhead() const { return mMode == LABELS && mRandomized && mState == EXHAUST; }
  /// the arguments of GetBunchLabels' gather of that next bunch, for a launch the caller enqueues on the COMPUTE
  /// stream before anything else touches the cache (the step's last weight update carries it); advances past
  /// that bunch
  BunchGather AheadGather(CuMatrix<BaseFloat>& rFeatures, CuVector<int>& rLabels);

  bool Full() { return mState == FULL; }
  bool Empty() { return mState == EMPTY || mIntakePos < mBunchsize; }
  int Discarded() { return mDiscarded; }
  void Trace(int trace) { mTrace = trace; }
  size_t IntakePos() const { return mIntakePos; }
  size_t Bunchsize() const { return mBunchsize; }
  size_t Cachesize() const { return mCachesize; }
  /// Re-arm the exhausted cache for another pass over the same intake (benchmark replay)
  void Rewind();
  /// host copy of the current permutation (tests)
  const std::vector<int>& Permutation() const { return mPermHost; }

 private:
  enum Mode { UNSET, DENSE, LABELS };
  void Alloc(size_t cols, size_t tcols);
  void BeginIntake();
  void CheckMode(Mode m);
  void WarnLong(size_t rows);
  void AdvanceAfterBunch();
  void EnterExhaust();
  void CopyAfterCompute();

  State mState = EMPTY;
  Mode mMode = UNSET;
  size_t mIntakePos = 0, mExhaustPos = 0, mCachesize = 0, mBunchsize = 0;
  int mDiscarded = 0;
  bool mRandomized = false;
  int mTrace = 0;
  Rng48* mRng = nullptr;

  CuMatrix<BaseFloat> mFeatures, mDesired, mFeaturesLeftover, mDesiredLeftover;
  CuVector<int> mLabels, mLabelsLeftover;
  size_t mLeftoverRows = 0;
  bool mLeftoverOnCopy = false;  // the leftover rows were written on the copy stream (host intake)
  // double buffer: the fill being taken in / exhausted is mFeatures/mLabels/mDesired; the other one
  // holds the previous fill, which queued gathers may still read
  CuMatrix<BaseFloat> mFeaturesAlt, mDesiredAlt;
  CuVector<int> mLabelsAlt;
  int mCurId = 0;                    // physical buffer behind mFeatures (0/1)
  hipStream_t mCopy = nullptr;
  hipEvent_t mRel[2] = {nullptr, nullptr};  // compute stream: last gathers of buffer 0/1 enqueued
  bool mHasRel[2] = {false, false};
  hipEvent_t mFilled = nullptr;      // copy stream: intake copies of the current fill enqueued
  hipEvent_t mSync = nullptr;
  // permutation upload from pinned host memory (two slots: the host never waits for the GPU)
  int* mPermPinned[2] = {nullptr, nullptr};
  hipEvent_t mPermEv[2] = {nullptr, nullptr};
  bool mPermEvSet[2] = {false, false};
  int mPermSlot = 0;
  CuVector<int> mPerm;          // device permutation of intake rows
  std::vector<int> mPermHost;
  // the next pass's permutation, drawn ahead on a host thread from a copy of the trainer's private stream
  // (a 64 k-row shuffle is ~0.3 ms of host time, more than a fast step's queue lead: MLP3 steps take 68 us).
  // Taken only when the stream still stands where the copy started (nothing drew from it or reset it in
  // between) and the fill size matches: the permutation and the stream's state are then exactly what the
  // shuffle in Randomize would produce.  TNET_SHUFFLE_AHEAD=0: off.
  void JoinAhead();
  std::thread mAheadThread;
  std::vector<int> mAheadPerm;
  uint64_t mAheadFrom = 0, mAheadTo = 0;
  size_t mAheadN = 0;
  bool mAheadValid = false;
};

}  // namespace TNet
