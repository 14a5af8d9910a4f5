// curbm.cpp -- see curbm.h.
#include "curbm.h"

#include <sys/time.h>

#include <algorithm>
#include <cstring>

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

// ============================================================================== CuRbm
void CuRbm::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuRbm::Propagate");
  // Y = hb + X W ; sigmoid for Bernoulli hidden units (cuRbm.cc:15-23)
  TNET_SAFE_CALL(tnet_affine_fwd(X.pCUData(), X.Dim(), mLinearity.pCUData(), mLinearity.Dim(), mBias.pCUData(),
                                 Y.pCUData(), Y.Dim(), mHidType == BERNOULLI ? 1 : 0, S));
}

void CuRbm::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuRbm::Backpropagate");
  // buf = X .* y(1-y) (Bernoulli) or X ; Y = buf W^T (cuRbm.cc:27-38)
  const CuMatrix<BaseFloat>* e = &X;
  if (mHidType == BERNOULLI) {
    mBackpropErrBuf.Init(X.Rows(), X.Cols());
    CuMath<BaseFloat>::DiffSigmoid(mBackpropErrBuf, X, GetOutput());
    e = &mBackpropErrBuf;
  }
  TNET_SAFE_CALL(tnet_affine_bwd(e->pCUData(), e->Dim(), mLinearity.pCUData(), mLinearity.Dim(), nullptr, 0,
                                 Y.pCUData(), Y.Dim(), 0, S));
}

void CuRbm::Update() {
  // cuRbm.cc:42-97 ("new implementation"): the CuBiasedLinearity update with the hidden bias,
  // on the error through the hidden nonlinearity (recomputed because of the backprop stopper)
  const CuMatrix<BaseFloat>& E = GetErrorInput();
  if (mHidType == BERNOULLI) {
    mBackpropErrBuf.Init(E.Rows(), E.Cols());
    CuMath<BaseFloat>::DiffSigmoid(mBackpropErrBuf, E, GetOutput());
    UpdateFrom(GetInput(), mBackpropErrBuf);
  } else {
    UpdateFrom(GetInput(), E);
  }
}

void CuRbm::Propagate(const CuMatrix<BaseFloat>& visProbs, CuMatrix<BaseFloat>& hidProbs) {
  if (visProbs.Cols() != GetNInputs()) {
    std::ostringstream os;
    os << " Nonmatching input dim, needs:" << GetNInputs() << " got:" << visProbs.Cols() << "\n";
    Error(os.str());
  }
  hidProbs.Init(visProbs.Rows(), GetNOutputs());
  PropagateFnc(visProbs, hidProbs);
}

void CuRbm::Reconstruct(const CuMatrix<BaseFloat>& hidState, CuMatrix<BaseFloat>& visProbs) {
  CuProfileScope p("CuRbm::Reconstruct");
  // vis = vb + h W^T ; sigmoid for Bernoulli visible units (cuRbm.cc:117-128)
  visProbs.Init(hidState.Rows(), GetNInputs());
  TNET_SAFE_CALL(tnet_affine_fwd_t(hidState.pCUData(), hidState.Dim(), mLinearity.pCUData(), mLinearity.Dim(),
                                   mVisBias.pCUData(), visProbs.pCUData(), visProbs.Dim(),
                                   mVisType == BERNOULLI ? 1 : 0, S));
}

void CuRbm::RbmUpdate(const CuMatrix<BaseFloat>& pos_vis, const CuMatrix<BaseFloat>& pos_hid,
                      const CuMatrix<BaseFloat>& neg_vis, const CuMatrix<BaseFloat>& neg_hid) {
  CuProfileScope p("CuRbm::RbmUpdate");
  // Generic (unstacked) form of cuRbm.cc:133-174, same operation order as the reference:
  //   corr = -lr/N neg_v^T neg_h + mmt corr ; corr += lr/N pos_v^T pos_h ; corr += -lr wc W ;
  //   W += corr ; biases likewise.  CuRbmTrainer uses the stacked one-GEMM form instead.
  if (!(pos_vis.Rows() == pos_hid.Rows() && pos_vis.Rows() == neg_vis.Rows() && pos_vis.Rows() == neg_hid.Rows() &&
        pos_vis.Cols() == neg_vis.Cols() && pos_hid.Cols() == neg_hid.Cols() && pos_vis.Cols() == GetNInputs() &&
        pos_hid.Cols() == GetNOutputs()))
    Error("CuRbm::RbmUpdate: non-matching dimensions");
  const BaseFloat N = (BaseFloat)pos_vis.Rows();
  const BaseFloat lr = mLearningRate;
  mLinearityCorrection.Gemm('T', 'N', -lr / N, neg_vis, neg_hid, mMomentum);
  mLinearityCorrection.Gemm('T', 'N', +lr / N, pos_vis, pos_hid, 1.0f);
  mLinearityCorrection.AddScaled(-lr * mWeightcost, mLinearity, 1.0f);
  mLinearity.AddScaled(1.0f, mLinearityCorrection, 1.0f);
  mVisBiasCorrection.AddColSum(-lr / N, neg_vis, mMomentum);
  mVisBiasCorrection.AddColSum(+lr / N, pos_vis, 1.0f);
  mVisBias.AddScaled(1.0f, mVisBiasCorrection, 1.0f);
  mBiasCorrection.AddColSum(-lr / N, neg_hid, mMomentum);
  mBiasCorrection.AddColSum(+lr / N, pos_hid, 1.0f);
  mBias.AddScaled(1.0f, mBiasCorrection, 1.0f);
}

void CuRbm::ReadFromStream(std::istream& rIn) {
  // "bern|gauss bern|gauss" then W^T [n_hid x n_vis], visible bias, hidden bias (cuRbm.cc:179-213)
  std::string str;
  rIn >> std::ws >> str;
  if (str == "bern") mVisType = BERNOULLI;
  else if (str == "gauss") mVisType = GAUSSIAN;
  else Error(std::string("Invalid unit type: ") + str);
  rIn >> std::ws >> str;
  if (str == "bern") mHidType = BERNOULLI;
  else if (str == "gauss") mHidType = GAUSSIAN;
  else Error(std::string("Invalid unit type: ") + str);
  BfMatrix transpose;
  ReadMatrixFast(rIn, transpose);
  if (transpose.Rows() != GetNOutputs() || transpose.Cols() != GetNInputs())
    Error("Wrong dimensionalities of the <rbm> matrix in network file");
  mLinearity.CopyFrom(BfMatrix(transpose, TRANS));
  BfVector bias;
  ReadVectorFast(rIn, bias);
  if (bias.Dim() != GetNInputs()) Error("Wrong dimensionality of the <rbm> visible bias");
  mVisBias.CopyFrom(bias);
  ReadVectorFast(rIn, bias);
  if (bias.Dim() != GetNOutputs()) Error("Wrong dimensionality of the <rbm> hidden bias");
  mBias.CopyFrom(bias);
}

void CuRbm::WriteToStream(std::ostream& rOut) {
  rOut << (mVisType == BERNOULLI ? " bern " : " gauss ");
  rOut << (mHidType == BERNOULLI ? " bern\n" : " gauss\n");
  BfMatrix tmp;
  mLinearity.CopyTo(tmp);
  rOut << BfMatrix(tmp, TRANS);
  BfVector vec;
  mVisBias.CopyTo(vec);
  rOut << vec << std::endl;
  mBias.CopyTo(vec);
  rOut << vec << std::endl;
}

// ============================================================================== CuRand
void CuRandState::SeedGpu(size_t rows, size_t cols, Rng48& rng) {
  std::vector<unsigned> host(rows * cols);
  for (int k = 0; k < 4; k++) {
    for (size_t i = 0; i < rows * cols; i++) {
      unsigned v = 0;
      while (v <= 128) v = (unsigned)rng.Lrand48();  // curand.tcc:39-41
      host[i] = v;
    }
    z[k].Init(rows, cols);
    z[k].CopyFromHost(host.data(), rows, cols, cols);
  }
}

void CuRandState::Check(const CuMatrix<BaseFloat>& m) const {
  if (m.Rows() != z[0].Rows() || m.Cols() != z[0].Cols() || m.Stride() != z[0].Stride())
    Error("CuRand: Non matching dims!!");
}

void CuRandState::Rand(CuMatrix<BaseFloat>& tgt) {
  tgt.Init(z[0].Rows(), z[0].Cols());
  Check(tgt);
  TNET_SAFE_CALL(tnetF_rand(tgt.pCUData(), tgt.Dim(), z[0].pCUData(), z[1].pCUData(), z[2].pCUData(),
                            z[3].pCUData(), S));
}

void CuRandState::GaussRand(CuMatrix<BaseFloat>& tgt) {
  tgt.Init(z[0].Rows(), z[0].Cols());
  Check(tgt);
  TNET_SAFE_CALL(tnetF_gauss_rand(tgt.pCUData(), tgt.Dim(), z[0].pCUData(), z[1].pCUData(), z[2].pCUData(),
                                  z[3].pCUData(), S));
}

void CuRandState::BinarizeProbs(const CuMatrix<BaseFloat>& probs, CuMatrix<BaseFloat>& states) {
  Check(probs);
  states.Init(z[0].Rows(), z[0].Cols());
  TNET_SAFE_CALL(tnet_rand_binarize(states.pCUData(), (int)states.Stride(), probs.pCUData(), probs.Dim(),
                                    z[0].pCUData(), z[1].pCUData(), z[2].pCUData(), z[3].pCUData(), S));
}

void CuRandState::AffineSigmoidSample(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& W,
                                      const CuVector<BaseFloat>& b, CuMatrix<BaseFloat>& probs,
                                      CuMatrix<BaseFloat>& states) {
  Check(probs);
  states.Init(z[0].Rows(), z[0].Cols());
  TNET_SAFE_CALL(tnet_affine_fwd_sample(X.pCUData(), X.Dim(), W.pCUData(), W.Dim(), b.pCUData(), probs.pCUData(),
                                        probs.Dim(), states.pCUData(), (int)states.Stride(), z[0].pCUData(),
                                        z[1].pCUData(), z[2].pCUData(), z[3].pCUData(), S));
}

void CuRandState::AddGaussNoise(CuMatrix<BaseFloat>& tgt, BaseFloat gscale) {
  Check(tgt);
  TNET_SAFE_CALL(tnet_add_gauss_noise(tgt.pCUData(), tgt.Dim(), gscale, z[0].pCUData(), z[1].pCUData(),
                                      z[2].pCUData(), z[3].pCUData(), S));
}

// ======================================================================= CuRbmTrainer
CuRbmTrainer::CuRbmTrainer(CuRbm* rbm, const RbmTrainerOptions& opt) : mRbm(rbm), mOpt(opt) {
  if (mOpt.bunchsize == 0) Error("CuRbmTrainer: bunchsize must be > 0");
  mOpt.cachesize = (mOpt.cachesize / mOpt.bunchsize) * mOpt.bunchsize;
  if (mOpt.cachesize == 0) Error("CuRbmTrainer: cachesize smaller than bunchsize");
  long seed = mOpt.seed;
  if (seed == 0) {
    struct timeval tv;
    gettimeofday(&tv, 0);
    seed = (int)(tv.tv_sec) + (int)tv.tv_usec;
  }
  // TRbmCu.cc:260-264: srand48(seed); CuRand(bunch, n_hid) draws its seeds first, the cache
  // shuffles continue on the same stream
  mRng.Seed(seed);
  const size_t B = mOpt.bunchsize, V = mRbm->GetNInputs(), H = mRbm->GetNOutputs();
  mRand.SeedGpu(B, H, mRng);
  mCache.Init(mOpt.cachesize, B);
  mCache.SetRng(&mRng);
  mCache.Trace(mOpt.trace);
  mVB[0].Init(2 * B, V);
  mVB[1].Init(2 * B, V);
  mH.Init(2 * B, H);
  mStates.Init(B, H);
  ViewV();
  CuMatrix<BaseFloat>::MakeView(mPosHid, mH.pCUData(), B, H, mH.Stride());
  CuMatrix<BaseFloat>::MakeView(mNegHid, mH.pCURowData(B), B, H, mH.Stride());
}

void CuRbmTrainer::ViewV() {
  const size_t B = mOpt.bunchsize, V = mRbm->GetNInputs();
  CuMatrix<BaseFloat>& cur = mVB[mCurV];
  CuMatrix<BaseFloat>& nxt = mVB[mCurV ^ 1];
  CuMatrix<BaseFloat>::MakeView(mPosVis, cur.pCUData(), B, V, cur.Stride());
  CuMatrix<BaseFloat>::MakeView(mNegVis, cur.pCURowData(B), B, V, cur.Stride());
  CuMatrix<BaseFloat>::MakeView(mNextPosVis, nxt.pCUData(), B, V, nxt.Stride());
}

void CuRbmTrainer::Step() {
  const size_t B = mOpt.bunchsize;
  CuRbm& rbm = *mRbm;
  const bool hid_bern = rbm.HidType() == CuRbm::BERNOULLI;
  // positive phase: pos_vis (gathered from the shuffled cache -- by the previous step's last launch when
  // that one carried it), pos_hid = p(h | v)
  if (mAheadV) {
    mCurV ^= 1;
    mAheadV = false;
    ViewV();
  } else {
    mCache.GetBunchLabels(mPosVis, mDummyLabels);
  }
  const CuMatrix<BaseFloat>& vs = mVB[mCurV];  // [pos_vis; neg_vis]
  // sample the hidden layer (TRbmCu.cc:336-341): Bernoulli units are sampled by the positive-phase
  // GEMM's own workgroups up to 2^20 units a bunch (bunch 256 x 2048: 62.1 -> 60.9 us a step); above,
  // the 32 B of generator state per unit make the sampling HBM-bound and the separate launch is as
  // fast (bunch 1024: 133.0 vs 138.2 us fused).  TNET_RBM_FUSED_SAMPLE=0 / 1 forces either form.
  static const char* fenv = getenv("TNET_RBM_FUSED_SAMPLE");
  const bool fused = fenv ? fenv[0] != '0' : B * rbm.GetNOutputs() <= (size_t)1 << 20;
  if (hid_bern && fused) {
    mRand.AffineSigmoidSample(mPosVis, rbm.VisHid(), rbm.HidBias(), mPosHid, mStates);
  } else if (hid_bern) {
    TNET_SAFE_CALL(tnet_affine_fwd(mPosVis.pCUData(), mPosVis.Dim(), rbm.VisHid().pCUData(), rbm.VisHid().Dim(),
                                   rbm.HidBias().pCUData(), mPosHid.pCUData(), mPosHid.Dim(), 1, S));
    mRand.BinarizeProbs(mPosHid, mStates);
  } else {
    TNET_SAFE_CALL(tnet_affine_fwd(mPosVis.pCUData(), mPosVis.Dim(), rbm.VisHid().pCUData(), rbm.VisHid().Dim(),
                                   rbm.HidBias().pCUData(), mPosHid.pCUData(), mPosHid.Dim(), 0, S));
    mStates.CopyFrom(mPosHid);
    mRand.AddGaussNoise(mStates);
  }
  // reconstruction, then the negative phase stored negated in rows B..2B-1 of mH
  TNET_SAFE_CALL(tnet_affine_fwd_t(mStates.pCUData(), mStates.Dim(), rbm.VisHid().pCUData(), rbm.VisHid().Dim(),
                                   rbm.VisBias().pCUData(), mNegVis.pCUData(), mNegVis.Dim(),
                                   rbm.VisType() == CuRbm::BERNOULLI ? 1 : 0, S));
  TNET_SAFE_CALL(tnet_affine_fwd(mNegVis.pCUData(), mNegVis.Dim(), rbm.VisHid().pCUData(), rbm.VisHid().Dim(),
                                 rbm.HidBias().pCUData(), mNegHid.pCUData(), mNegHid.Dim(), hid_bern ? 3 : 2, S));
  // CD-1 update (cuRbm.cc:133-174): one GEMM over the stacked statistics + two signed colsums; both
  // bias updates and the reconstruction error (mse.Evaluate(neg_vis, pos_vis), TRbmCu.cc:350) in one
  // launch over the stacked statistics -- and where the GEMM runs the 64x64 tiles unsplit (bunch 256),
  // that launch and the GEMM's are one (tnet_rbm_update_stats: the statistics blocks beside the tiles)
  // The next shuffled bunch of the fill is gathered into the other visible buffer by this last launch, on
  // CUs beside the update's tiles (tnet_rbm_update_stats_gather; TNET_GATHER_TAIL=0: a gather launch at the
  // start of the next step); where that launch is declined the gather follows the step.  Up to bunch 512:
  // at bunch 256 4.19 M -> 4.25-4.44 M frames/s, at 1024 8.22 M -> 8.12 M (the 1024-row gather holds back the
  // statistics blocks queued behind it; profiles/r03_gather_tail_ab.json), so larger bunches keep the
  // separate gather launch.
  const float lr = rbm.LearnRate(), scale = lr / (float)B;
  static const bool tail = !(getenv("TNET_GATHER_TAIL") && getenv("TNET_GATHER_TAIL")[0] == '0');
  BunchGather tg;
  const bool tail_now = tail && B <= 512 && mCache.HasBunchAhead();
  // once the cache has moved past the next bunch it must land in the other buffer whatever happens below
  // (ADVICE r3): mAheadV is set at once, and if the step throws before the gather went out, the guard
  // launches it (unchecked) while unwinding
  struct Pending {
    const BunchGather* g = nullptr;
    hipStream_t s = nullptr;
    ~Pending() {
      if (g) (void)tnet_gather_bunch(g->y, g->x, g->labels_out, g->labels_in, g->copy_from, g->dy, g->dx, s);
    }
  } pending;
  if (tail_now) {
    tg = mCache.AheadGather(mNextPosVis, mDummyLabels);
    mAheadV = true;
    pending.g = &tg;
    pending.s = (hipStream_t)S;
  }
  auto finish_gather = [&](bool done) {
    if (!tail_now) return;
    pending.g = nullptr;
    if (!done)
      TNET_SAFE_CALL(tnet_gather_bunch(tg.y, tg.x, tg.labels_out, tg.labels_in, tg.copy_from, tg.dy, tg.dx, S));
  };
  int st = TNET_ERR_UNSUPPORTED;
  if (tail_now) {
    st = tnet_rbm_update_stats_gather(
        vs.pCUData(), vs.Dim(), mH.pCUData(), mH.Dim(), rbm.VisHid().pCUData(), rbm.VisHid().Dim(),
        rbm.VisHidCorrection().pCUData(), (int)rbm.VisHidCorrection().Stride(), scale, rbm.Momentum(),
        -lr * rbm.Weightcost(), (int)B, rbm.VisBias().pCUData(), rbm.VisBiasCorrection().pCUData(),
        rbm.HidBias().pCUData(), rbm.HidBiasCorrection().pCUData(), mMse.DeviceStats(), tg.y, tg.x, tg.labels_out,
        tg.labels_in, tg.copy_from, tg.dy, tg.dx, S);
    if (st == TNET_OK) {
      finish_gather(true);
      mMse.AddFrames(B);
      if (mOpt.trace & 2) std::cout << "." << std::flush;
      mSteps++;
      return;
    }
  }
  if (st == TNET_ERR_UNSUPPORTED)
    st = tnet_rbm_update_stats(vs.pCUData(), vs.Dim(), mH.pCUData(), mH.Dim(), rbm.VisHid().pCUData(),
                               rbm.VisHid().Dim(), rbm.VisHidCorrection().pCUData(),
                               (int)rbm.VisHidCorrection().Stride(), scale, rbm.Momentum(), -lr * rbm.Weightcost(),
                               (int)B, rbm.VisBias().pCUData(), rbm.VisBiasCorrection().pCUData(),
                               rbm.HidBias().pCUData(), rbm.HidBiasCorrection().pCUData(), mMse.DeviceStats(), S);
  if (st == TNET_OK) {
    finish_gather(false);
    mMse.AddFrames(B);
    if (mOpt.trace & 2) std::cout << "." << std::flush;
    mSteps++;
    return;
  }
  if (st != TNET_ERR_UNSUPPORTED) TNET_SAFE_CALL(st);
  TNET_SAFE_CALL(tnet_rbm_update(vs.pCUData(), vs.Dim(), mH.pCUData(), mH.Dim(), rbm.VisHid().pCUData(),
                                 rbm.VisHid().Dim(), rbm.VisHidCorrection().pCUData(),
                                 (int)rbm.VisHidCorrection().Stride(), scale, rbm.Momentum(), -lr * rbm.Weightcost(),
                                 S));
  st = tnet_rbm_stats_update(vs.pCUData(), vs.Dim(), mH.pCUData(), mH.Dim(), (int)B, rbm.VisBias().pCUData(),
                             rbm.VisBiasCorrection().pCUData(), rbm.HidBias().pCUData(),
                             rbm.HidBiasCorrection().pCUData(), scale, rbm.Momentum(), mMse.DeviceStats(), S);
  if (st == TNET_ERR_UNSUPPORTED) {  // bunches above 4096 frames: the two column sums + the MSE kernel
    void* ws = CuDevice::Instantiate().Workspace(
        (size_t)std::max(tnet_col_sum_workspace(vs.Dim()), tnet_col_sum_workspace(mH.Dim())));
    TNET_SAFE_CALL(tnet_rbm_bias_update(vs.pCUData(), vs.Dim(), (int)B, rbm.VisBias().pCUData(),
                                        rbm.VisBiasCorrection().pCUData(), scale, rbm.Momentum(), ws, S));
    TNET_SAFE_CALL(tnet_rbm_bias_update(mH.pCUData(), mH.Dim(), (int)(2 * B), rbm.HidBias().pCUData(),
                                        rbm.HidBiasCorrection().pCUData(), scale, rbm.Momentum(), ws, S));
    mMse.EvaluateStats(mNegVis, mPosVis);
  } else {
    TNET_SAFE_CALL(st);
    mMse.AddFrames(B);
  }
  finish_gather(false);
  if (mOpt.trace & 2) std::cout << "." << std::flush;
  mSteps++;
}

void CuRbmTrainer::DrainCache() {
  if (mOpt.randomize) mCache.Randomize();
  while (mAheadV || !mCache.Empty()) Step();
  mTrainedSinceFill = true;
}

void CuRbmTrainer::AddUtterance(const float* feats, size_t rows, size_t cols, size_t ld) {
  if (cols != mRbm->GetNInputs()) Error("CuRbmTrainer::AddUtterance: feature dim != RBM visible dim");
  if (rows == 0) return;
  if (mZeroLabels.size() < rows) mZeroLabels.assign(rows, 0);  // "fake the labels" (TRbmCu.cc:311)
  mCache.AddDataHost(feats, rows, cols, ld, mZeroLabels.data());
  mTrainedSinceFill = false;
  if (mCache.Full()) DrainCache();
}

void CuRbmTrainer::Finish() {
  if (!mTrainedSinceFill && mCache.IntakePos() > 0) DrainCache();
}

size_t CuRbmTrainer::Prefill(const float* feats, size_t rows, size_t cols, size_t ld) {
  if (mCache.Full()) return 0;
  const size_t space = mOpt.cachesize - mCache.IntakePos();
  const size_t take = rows < space ? rows : space;
  if (mZeroLabels.size() < take) mZeroLabels.assign(take, 0);
  mCache.AddDataHost(feats, take, cols, ld, mZeroLabels.data());
  if (mCache.Full() && mOpt.randomize) mCache.Randomize();
  return take;
}

void CuRbmTrainer::Replay(long n) {
  for (long i = 0; i < n; i++) {
    if (!mAheadV && mCache.Empty()) {
      mCache.Rewind();
      if (mOpt.randomize) mCache.Randomize();
    }
    Step();
  }
}

}  // namespace TNet
