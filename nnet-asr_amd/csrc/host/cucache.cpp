// cucache.cpp -- see cucache.h.  State machine follows src/CuTNetLib/cuCache.cc:22-200.
#include "cucache.h"

#include <cstdlib>
#include <numeric>

namespace TNet {

Rng48& GlobalRng() {
  static Rng48 rng(0);
#ifdef TNET_HOST_KALDILIB
  static bool libc = (rng.UseLibc(true), true);  // the reference drivers seed libc's srand48
  (void)libc;
#endif
  return rng;
}
void SeedRandom(long seed) { GlobalRng().Seed(seed); }

#define S ((void*)CuDevice::Instantiate().Stream())

CuCache::CuCache() {}
CuCache::~CuCache() {
  JoinAhead();
  if (mCopy) (void)hipStreamSynchronize(mCopy);
  (void)hipStreamSynchronize(CuDevice::Instantiate().Stream());
  for (hipEvent_t e : {mRel[0], mRel[1], mFilled, mSync, mPermEv[0], mPermEv[1]})
    if (e) (void)hipEventDestroy(e);
  for (int* p : mPermPinned)
    if (p) (void)hipHostFree(p);
  if (mCopy) (void)hipStreamDestroy(mCopy);
}

// the copy stream waits for everything enqueued on the compute stream so far
void CuCache::CopyAfterCompute() {
  TNET_HIP_CALL(hipEventRecord(mSync, CuDevice::Instantiate().Stream()));
  TNET_HIP_CALL(hipStreamWaitEvent(mCopy, mSync, 0));
}

// the compute stream waits for everything enqueued on the copy stream so far
static void compute_after_copy(hipStream_t copy, hipEvent_t ev) {
  TNET_HIP_CALL(hipEventRecord(ev, copy));
  TNET_HIP_CALL(hipStreamWaitEvent(CuDevice::Instantiate().Stream(), ev, 0));
}

// first bunch of a fill: the compute stream waits for the fill's intake copies
void CuCache::EnterExhaust() {
  mState = EXHAUST;
  mExhaustPos = 0;
  TNET_HIP_CALL(hipEventRecord(mFilled, mCopy));
  TNET_HIP_CALL(hipStreamWaitEvent(CuDevice::Instantiate().Stream(), mFilled, 0));
}

void CuCache::Init(size_t cachesize, size_t bunchsize) {
  if (bunchsize == 0 || (cachesize % bunchsize) != 0) Error("Non divisible cachesize by bunchsize");
  mCachesize = cachesize;
  mBunchsize = bunchsize;
  mState = EMPTY;
  mIntakePos = 0;
  mExhaustPos = 0;
  mRandomized = false;
}

void CuCache::CheckMode(Mode m) {
  if (mMode == UNSET) mMode = m;
  if (mMode != m) Error("CuCache: mixing dense targets and class-id targets");
}

void CuCache::WarnLong(size_t rows) {
  if (rows > mCachesize / 2) {
    std::ostringstream os;
    os << "Too long segment and small feature cache!  cachesize: " << mCachesize << " segmentsize: " << rows;
    Warning(os.str());
  }
}

void CuCache::Alloc(size_t cols, size_t tcols) {
  if (!mCopy) {
    TNET_HIP_CALL(hipStreamCreateWithFlags(&mCopy, hipStreamNonBlocking));
    for (hipEvent_t* e : {&mRel[0], &mRel[1], &mFilled, &mSync, &mPermEv[0], &mPermEv[1]})
      TNET_HIP_CALL(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  if (mPerm.Dim() != mCachesize) {
    // sized once: a reallocation could hand memory that queued gathers still read to someone else
    (void)hipStreamSynchronize(CuDevice::Instantiate().Stream());
    mPerm.Init(mCachesize);
    for (int k = 0; k < 2; ++k) {
      if (mPermPinned[k]) TNET_HIP_CALL(hipHostFree(mPermPinned[k]));
      TNET_HIP_CALL(hipHostMalloc((void**)&mPermPinned[k], mCachesize * sizeof(int), hipHostMallocDefault));
      mPermEvSet[k] = false;
    }
  }
  // a shape change re-Inits buffers that gathers (compute stream) or intake copies (copy stream)
  // of the previous fill may still use; the blocks go back to CuDevice's pool, which assumes all
  // work on them is ordered on the compute stream -- drain both streams first
  const bool resize = (mFeatures.Rows() > 0 && (mFeatures.Rows() != mCachesize || mFeatures.Cols() != cols)) ||
                      (mMode == DENSE && mDesired.Rows() > 0 &&
                       (mDesired.Rows() != mCachesize || mDesired.Cols() != tcols)) ||
                      (mMode != DENSE && mLabels.Dim() > 0 && mLabels.Dim() != mCachesize);
  if (resize) {
    TNET_HIP_CALL(hipStreamSynchronize(mCopy));
    TNET_HIP_CALL(hipStreamSynchronize(CuDevice::Instantiate().Stream()));
  }
  bool fresh = false;
  auto mat = [&](CuMatrix<BaseFloat>& m, size_t c) {
    if (m.Rows() != mCachesize || m.Cols() != c) {
      m.Init(mCachesize, c);
      fresh = true;
    }
  };
  auto vec = [&](CuVector<int>& v) {
    if (v.Dim() != mCachesize) {
      v.Init(mCachesize);
      fresh = true;
    }
  };
  mat(mFeatures, cols);
  mat(mFeaturesAlt, cols);
  mat(mFeaturesLeftover, cols);
  if (mMode == DENSE) {
    mat(mDesired, tcols);
    mat(mDesiredAlt, tcols);
    mat(mDesiredLeftover, tcols);
  } else {
    vec(mLabels);
    vec(mLabelsAlt);
    vec(mLabelsLeftover);
  }
  if (fresh) CopyAfterCompute();  // the allocations' zero-fills (compute stream) precede any copy
}

void CuCache::BeginIntake() {
  if (mState != EMPTY) return;
  if (mTrace & 3) std::cout << "/" << std::flush;
  mState = INTAKE;
  mIntakePos = 0;
  // flip the double buffer: the fill just exhausted (its gathers are all enqueued) becomes the
  // alternate; the new fill goes into the buffer the fill before last used, once its gathers ran
  hipStream_t cs = CuDevice::Instantiate().Stream();
  TNET_HIP_CALL(hipEventRecord(mRel[mCurId], cs));
  mHasRel[mCurId] = true;
  mFeatures.Swap(mFeaturesAlt);
  mDesired.Swap(mDesiredAlt);
  mLabels.Swap(mLabelsAlt);
  mCurId ^= 1;
  if (mHasRel[mCurId]) TNET_HIP_CALL(hipStreamWaitEvent(mCopy, mRel[mCurId], 0));
  size_t leftover = mLeftoverRows;
  if (leftover > mCachesize) {
    std::ostringstream os;
    os << "Too small feature cache: " << mCachesize << ", truncating: " << leftover - mCachesize
       << " frames from previous segment leftover";
    Warning(os.str());
    leftover = mCachesize;
  }
  if (leftover > 0) {
    // on the copy stream; leftover rows a device intake wrote on the compute stream are waited for
    if (!mLeftoverOnCopy) CopyAfterCompute();
    TNET_HIP_CALL(hipMemcpy2DAsync(mFeatures.pCUData(), mFeatures.Stride() * sizeof(float), mFeaturesLeftover.pCUData(),
                                   mFeaturesLeftover.Stride() * sizeof(float), mFeatures.Cols() * sizeof(float),
                                   leftover, hipMemcpyDeviceToDevice, mCopy));
    if (mMode == DENSE) {
      TNET_HIP_CALL(hipMemcpy2DAsync(mDesired.pCUData(), mDesired.Stride() * sizeof(float), mDesiredLeftover.pCUData(),
                                     mDesiredLeftover.Stride() * sizeof(float), mDesired.Cols() * sizeof(float),
                                     leftover, hipMemcpyDeviceToDevice, mCopy));
    } else {
      TNET_HIP_CALL(hipMemcpyAsync(mLabels.pCUData(), mLabelsLeftover.pCUData(), leftover * sizeof(int),
                                   hipMemcpyDeviceToDevice, mCopy));
    }
    mIntakePos += leftover;
  }
  mLeftoverRows = 0;
  // an utterance whose leftover alone fills the cache leaves no space for the next one: the
  // reference asserts here (cuCache.cc:97 assert(cache_space > 0), Cache.cc:117 on the CPU)
  if (mIntakePos >= mCachesize)
    Error("CuCache: the previous segment's leftover fills the whole cache (cache smaller than the longest "
          "utterance; the reference asserts cache_space > 0, cuCache.cc:97)");
}

void CuCache::AddData(const CuMatrix<BaseFloat>& rFeatures, const CuMatrix<BaseFloat>& rDesired) {
  if (rFeatures.Rows() != rDesired.Rows()) Error("CuCache::AddData: rows of features != rows of targets");
  CheckMode(DENSE);
  Alloc(rFeatures.Cols(), rDesired.Cols());
  WarnLong(rFeatures.Rows());
  BeginIntake();
  if (mState != INTAKE) Error("CuCache::AddData: cache not in INTAKE state");
  if (mTrace & 2) std::cout << "F" << std::flush;
  const size_t space = mCachesize - mIntakePos, len = rFeatures.Rows();
  const size_t fill = space < len ? space : len, leftover = len - fill;
  mFeatures.CopyRows(fill, 0, rFeatures, mIntakePos);
  mDesired.CopyRows(fill, 0, rDesired, mIntakePos);
  if (leftover > 0) {
    // the leftover buffers hold the cache size (the reference truncates a longer leftover); the copy
    // stream may still be reading the previous leftover
    const size_t keep = leftover < mCachesize ? leftover : mCachesize;
    compute_after_copy(mCopy, mSync);
    mFeaturesLeftover.CopyRows(keep, fill, rFeatures, 0);
    mDesiredLeftover.CopyRows(keep, fill, rDesired, 0);
    mLeftoverRows = leftover;
    mLeftoverOnCopy = false;
  }
  mIntakePos += fill;
  if (mIntakePos == mCachesize) {
    if (mTrace & 3) std::cout << "\\" << std::flush;
    mState = FULL;
  }
}

void CuCache::AddDataLabels(const CuMatrix<BaseFloat>& rFeatures, const CuVector<int>& rLabels) {
  if (rFeatures.Rows() != rLabels.Dim()) Error("CuCache::AddDataLabels: rows of features != number of labels");
  CheckMode(LABELS);
  Alloc(rFeatures.Cols(), 0);
  WarnLong(rFeatures.Rows());
  BeginIntake();
  if (mState != INTAKE) Error("CuCache::AddDataLabels: cache not in INTAKE state");
  const size_t space = mCachesize - mIntakePos, len = rFeatures.Rows();
  const size_t fill = space < len ? space : len, leftover = len - fill;
  hipStream_t st = CuDevice::Instantiate().Stream();
  mFeatures.CopyRows(fill, 0, rFeatures, mIntakePos);
  TNET_HIP_CALL(hipMemcpyAsync(mLabels.pCUData() + mIntakePos, rLabels.pCUData(), fill * sizeof(int),
                               hipMemcpyDeviceToDevice, st));
  if (leftover > 0) {
    const size_t keep = leftover < mCachesize ? leftover : mCachesize;
    compute_after_copy(mCopy, mSync);
    mFeaturesLeftover.CopyRows(keep, fill, rFeatures, 0);
    TNET_HIP_CALL(hipMemcpyAsync(mLabelsLeftover.pCUData(), rLabels.pCUData() + fill, keep * sizeof(int),
                                 hipMemcpyDeviceToDevice, st));
    mLeftoverRows = leftover;
    mLeftoverOnCopy = false;
  }
  mIntakePos += fill;
  if (mIntakePos == mCachesize) mState = FULL;
}

void CuCache::AddDataHost(const float* feats, size_t rows, size_t cols, size_t ld, const int* labels) {
  CheckMode(LABELS);
  Alloc(cols, 0);
  WarnLong(rows);
  BeginIntake();
  if (mState != INTAKE) Error("CuCache::AddDataHost: cache not in INTAKE state");
  const size_t space = mCachesize - mIntakePos;
  const size_t fill = space < rows ? space : rows, leftover = rows - fill;
  hipStream_t st = mCopy;  // overlaps the training queued on the compute stream
  if (fill) {
    TNET_HIP_CALL(hipMemcpy2DAsync(mFeatures.pCURowData(mIntakePos), mFeatures.Stride() * sizeof(float), feats,
                                   ld * sizeof(float), cols * sizeof(float), fill, hipMemcpyHostToDevice, st));
    TNET_HIP_CALL(hipMemcpyAsync(mLabels.pCUData() + mIntakePos, labels, fill * sizeof(int), hipMemcpyHostToDevice, st));
  }
  if (leftover > 0) {
    const size_t keep = leftover < mCachesize ? leftover : mCachesize;
    TNET_HIP_CALL(hipMemcpy2DAsync(mFeaturesLeftover.pCUData(), mFeaturesLeftover.Stride() * sizeof(float),
                                   feats + fill * ld, ld * sizeof(float), cols * sizeof(float), keep,
                                   hipMemcpyHostToDevice, st));
    TNET_HIP_CALL(hipMemcpyAsync(mLabelsLeftover.pCUData(), labels + fill, keep * sizeof(int),
                                 hipMemcpyHostToDevice, st));
    mLeftoverRows = leftover;
    mLeftoverOnCopy = true;
  }
  // the caller's host buffers may be reused: wait for the copies (not for the queued training)
  TNET_HIP_CALL(hipStreamSynchronize(st));
  mIntakePos += fill;
  if (mIntakePos == mCachesize) mState = FULL;
}

void CuCache::Randomize() {
  if (!(mState == FULL || mState == INTAKE)) Error("CuCache::Randomize: cache not filled");
  if (mTrace & 3) std::cout << "R" << std::flush;
  Rng48& rng = mRng ? *mRng : GlobalRng();
  JoinAhead();
  if (mAheadValid && mRng && !rng.Libc() && mAheadN == mIntakePos && rng.State() == mAheadFrom) {
    mPermHost.swap(mAheadPerm);  // drawn ahead from this very state (see cucache.h)
    rng.SetState(mAheadTo);
  } else {
    mPermHost.resize(mIntakePos);
    std::iota(mPermHost.begin(), mPermHost.end(), 0);
    rng.RandomShuffle(mPermHost.data(), mIntakePos);
  }
  mAheadValid = false;
  // upload from a pinned slot on the compute stream (ordered after the gathers that read the
  // previous permutation); the slot's previous upload finished long ago (two shuffles back)
  const int k = mPermSlot;
  if (mPermEvSet[k]) TNET_HIP_CALL(hipEventSynchronize(mPermEv[k]));
  std::copy(mPermHost.begin(), mPermHost.end(), mPermPinned[k]);
  hipStream_t cs = CuDevice::Instantiate().Stream();
  TNET_HIP_CALL(hipMemcpyAsync(mPerm.pCUData(), mPermPinned[k], mIntakePos * sizeof(int), hipMemcpyHostToDevice, cs));
  TNET_HIP_CALL(hipEventRecord(mPermEv[k], cs));
  mPermEvSet[k] = true;
  mPermSlot ^= 1;
  mRandomized = true;
  static const bool ahead = !(getenv("TNET_SHUFFLE_AHEAD") && getenv("TNET_SHUFFLE_AHEAD")[0] == '0');
  if (ahead && mRng && !rng.Libc()) {  // the process stream may have other users: never drawn ahead
    mAheadFrom = rng.State();
    mAheadN = mIntakePos;
    mAheadValid = true;
    mAheadThread = std::thread([this] {
      Rng48 r;
      r.SetState(mAheadFrom);
      mAheadPerm.resize(mAheadN);
      std::iota(mAheadPerm.begin(), mAheadPerm.end(), 0);
      r.RandomShuffle(mAheadPerm.data(), mAheadN);
      mAheadTo = r.State();
    });
  }
}

void CuCache::JoinAhead() {
  if (mAheadThread.joinable()) mAheadThread.join();
}

void CuCache::Rewind() {
  if (mIntakePos < mBunchsize) Error("CuCache::Rewind: nothing to replay");
  mState = FULL;
  mExhaustPos = 0;
}

void CuCache::AdvanceAfterBunch() {
  mExhaustPos += mBunchsize;
  if (mExhaustPos > mIntakePos - mBunchsize) {
    mDiscarded += (int)(mIntakePos - mExhaustPos);
    mState = EMPTY;
  }
}

void CuCache::GetBunch(CuMatrix<BaseFloat>& rFeatures, CuMatrix<BaseFloat>& rDesired) {
  if (mState == EMPTY) Error("GetBunch on empty cache!!!");
  if (mMode != DENSE) Error("CuCache::GetBunch: cache holds class ids, use GetBunchLabels");
  if (mState == FULL || mState == INTAKE) EnterExhaust();
  rFeatures.Init(mBunchsize, mFeatures.Cols());
  rDesired.Init(mBunchsize, mDesired.Cols());
  if (mRandomized) {
    TnetMatrixDim df = rFeatures.Dim(), dd = rDesired.Dim();
    TNET_SAFE_CALL(tnetF_randomize(rFeatures.pCUData(), mFeatures.pCUData(), mPerm.pCUData() + mExhaustPos, df,
                                   mFeatures.Dim(), S));
    TNET_SAFE_CALL(tnetF_randomize(rDesired.pCUData(), mDesired.pCUData(), mPerm.pCUData() + mExhaustPos, dd,
                                   mDesired.Dim(), S));
  } else {
    rFeatures.CopyRows(mBunchsize, mExhaustPos, mFeatures, 0);
    rDesired.CopyRows(mBunchsize, mExhaustPos, mDesired, 0);
  }
  AdvanceAfterBunch();
}

void CuCache::GetBunchLabels(CuMatrix<BaseFloat>& rFeatures, CuVector<int>& rLabels) {
  if (mState == EMPTY) Error("GetBunch on empty cache!!!");
  if (mMode != LABELS) Error("CuCache::GetBunchLabels: cache holds dense targets, use GetBunch");
  if (mState == FULL || mState == INTAKE) EnterExhaust();
  rFeatures.Init(mBunchsize, mFeatures.Cols());
  rLabels.Init(mBunchsize);
  if (mRandomized) {
    KTScope kt("gather", 2.0 * mBunchsize * mFeatures.Cols() * 4.0);
    TNET_SAFE_CALL(tnet_gather_bunch(rFeatures.pCUData(), mFeatures.pCUData(), rLabels.pCUData(), mLabels.pCUData(),
                                     mPerm.pCUData() + mExhaustPos, rFeatures.Dim(), mFeatures.Dim(), S));
  } else {
    rFeatures.CopyRows(mBunchsize, mExhaustPos, mFeatures, 0);
    TNET_HIP_CALL(hipMemcpyAsync(rLabels.pCUData(), mLabels.pCUData() + mExhaustPos, mBunchsize * sizeof(int),
                                 hipMemcpyDeviceToDevice, CuDevice::Instantiate().Stream()));
  }
  AdvanceAfterBunch();
}

BunchGather CuCache::AheadGather(CuMatrix<BaseFloat>& rFeatures, CuVector<int>& rLabels) {
  if (!HasBunchAhead()) Error("CuCache::AheadGather: no shuffled bunch ahead");
  if (rFeatures.Rows() != mBunchsize || rFeatures.Cols() != mFeatures.Cols() || rLabels.Dim() != mBunchsize)
    Error("CuCache::AheadGather: destination not sized for a bunch");
  BunchGather g;
  g.y = rFeatures.pCUData();
  g.x = mFeatures.pCUData();
  g.labels_out = rLabels.pCUData();
  g.labels_in = mLabels.pCUData();
  g.copy_from = mPerm.pCUData() + mExhaustPos;
  g.dy = rFeatures.Dim();
  g.dx = mFeatures.Dim();
  AdvanceAfterBunch();
  return g;
}

}  // namespace TNet
