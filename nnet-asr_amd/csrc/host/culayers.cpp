// culayers.cpp -- <biasedlinearity>, <sigmoid>, <softmax> on the fused gfx950 kernels.
#include "culayers.h"

#include "gradexchange.h"

#include <cctype>
#include <cstdlib>

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

// ------------------------------------------------------------------------------ text parsing
static bool next_token(std::streambuf* sb, char* buf, size_t cap) {
  int c = sb->sgetc();
  while (c != EOF && std::isspace(c)) c = sb->snextc();
  if (c == EOF) return false;
  size_t n = 0;
  while (c != EOF && !std::isspace(c)) {
    if (n + 1 < cap) buf[n++] = (char)c;
    c = sb->snextc();
  }
  buf[n] = 0;
  return true;
}

void ReadMatrixFast(std::istream& in, Matrix<BaseFloat>& m) {
  in >> std::ws;
  if (in.peek() != 'm') Error("Failed to read matrix from stream: expected 'm R C'");
  in.get();
  long long r = -1, c = -1;
  in >> r >> c;
  if (in.fail() || r < 0 || c < 0) Error("Failed to read matrix from stream: no size");
  m.Init((size_t)r, (size_t)c);
  std::streambuf* sb = in.rdbuf();
  char tok[128];
  for (long long i = 0; i < r; i++) {
    float* p = m.pRowData((size_t)i);  // rows may be padded (KaldiLib Matrix stride)
    for (long long j = 0; j < c; j++) {
      if (!next_token(sb, tok, sizeof tok)) Error("Failed to read matrix from stream: truncated");
      char* end = nullptr;
      p[j] = std::strtof(tok, &end);
      if (end == tok) Error(std::string("Failed to read matrix from stream: bad token ") + tok);
    }
  }
}

void ReadVectorFast(std::istream& in, Vector<BaseFloat>& v) {
  in >> std::ws;
  if (in.peek() != 'v') Error("Failed to read vector from stream: expected 'v N'");
  in.get();
  long long n = -1;
  in >> n;
  if (in.fail() || n < 0) Error("Failed to read vector from stream: no size");
  v.Init((size_t)n);
  std::streambuf* sb = in.rdbuf();
  char tok[128];
  for (long long i = 0; i < n; i++) {
    if (!next_token(sb, tok, sizeof tok)) Error("Failed to read vector from stream: truncated");
    char* end = nullptr;
    v[(size_t)i] = std::strtof(tok, &end);
    if (end == tok) Error(std::string("Failed to read vector from stream: bad token ") + tok);
  }
}

// ------------------------------------------------------------------------- CuBiasedLinearity
void CuBiasedLinearity::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuBiasedLinearity::Propagate");
  // Y = b + X W  (AddScaledRow + Gemm('N','N',1,X,W,1), cuBiasedLinearity.cc:11-16) in one kernel
  if (X.Rows() == 1) {  // single frame (TRecurrentCu): split-K row-vector kernel
    void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_gemv_workspace((int)GetNInputs(), (int)GetNOutputs()));
    TNET_SAFE_CALL(tnet_gemv_rowvec(X.pCUData(), (int)GetNInputs(), mLinearity.pCUData(), (int)mLinearity.Stride(),
                                    mBias.pCUData(), Y.pCUData(), (int)GetNOutputs(), 0, ws, S));
    return;
  }
  TNET_SAFE_CALL(tnet_affine_fwd(X.pCUData(), X.Dim(), mLinearity.pCUData(), mLinearity.Dim(), mBias.pCUData(),
                                 Y.pCUData(), Y.Dim(), 0, S));
}

void CuBiasedLinearity::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuProfileScope p("CuBiasedLinearity::Backpropagate");
  // Y = X W^T  (Gemm('N','T',1,E,W,0), cuBiasedLinearity.cc:21-25)
  if (X.Rows() == 1) {  // single frame: one wavefront per row of W
    TNET_SAFE_CALL(tnet_gemv_rows(mLinearity.pCUData(), (int)mLinearity.Stride(), 0, (int)GetNInputs(),
                                  (int)GetNOutputs(), X.pCUData(), Y.pCUData(), 0.0f, nullptr, S));
    return;
  }
  TNET_SAFE_CALL(tnet_affine_bwd(X.pCUData(), X.Dim(), mLinearity.pCUData(), mLinearity.Dim(), nullptr, 0,
                                 Y.pCUData(), Y.Dim(), 0, S));
}

void CuBiasedLinearity::UpdateConstants(size_t rows, float* scale, float* l2) const {
  // cuBiasedLinearity.cc:46-64
  BaseFloat N = 1;
  if (mGradDivFrm) N = static_cast<BaseFloat>(rows);
  BaseFloat mmt_gain = static_cast<BaseFloat>(1.0 / (1.0 - mMomentum));
  N *= mmt_gain;
  *scale = -mLearningRate / N;
  *l2 = -mLearningRate * mWeightcost * (mGradDivFrm ? 1.0f : (BaseFloat)rows);
}

void CuBiasedLinearity::UpdateFrom(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E) {
  CuProfileScope p("CuBiasedLinearity::Update");
  float scale, l2;
  UpdateConstants(X.Rows(), &scale, &l2);
  const bool mmt = mMomentum != 0.0f;
  if (X.Rows() == 1) {  // single frame (TRecurrentCu's output layer): one rank-1 launch
    TNET_SAFE_CALL(tnet_affine_update_row(X.pCUData(), (int)GetNInputs(), E.pCUData(), (int)GetNOutputs(),
                                          mLinearity.pCUData(), (int)mLinearity.Stride(),
                                          mmt ? mLinearityCorrection.pCUData() : nullptr,
                                          (int)mLinearityCorrection.Stride(), mBias.pCUData(),
                                          mmt ? mBiasCorrection.pCUData() : nullptr, scale, mMomentum, l2, S));
    mShadowValid = false;  // the rank-1 kernel writes W only
    return;
  }
  // bias first: it reads only E (the weight kernel rewrites W in place)
  TnetMatrixDim dE = E.Dim();
  void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_col_sum_workspace(dE));
  {
    KTScope kt("bias_update:" + std::to_string(GetNOutputs()), 4.0 * dE.rows * dE.cols);
    TNET_SAFE_CALL(tnet_bias_update(E.pCUData(), dE, mBias.pCUData(), mmt ? mBiasCorrection.pCUData() : nullptr,
                                    nullptr, scale, mMomentum, ws, S));
  }
  // corrW = X^T E + mmt corrW ; W += scale corrW ; W += l2 W   -- one GEMM with an SGD epilogue.
  // With momentum 0 the correction buffer is never read (momentum is fixed per run, TNetCu.cc:322),
  // so it is not written either.
  KTScope kt("gemm_upd:" + std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs()),
             2.0 * X.Rows() * GetNInputs() * GetNOutputs());
  TNET_SAFE_CALL(tnet_affine_update(X.pCUData(), X.Dim(), E.pCUData(), dE, mLinearity.pCUData(), mLinearity.Dim(),
                                    mmt ? mLinearityCorrection.pCUData() : nullptr,
                                    (int)mLinearityCorrection.Stride(), scale, mMomentum, l2, S));
  NoteUpdate();
}

void CuBiasedLinearity::UseShadow() {
  if (!mShadowOn || mLinearityT.Rows() != mLinearity.Cols() || mLinearityT.Cols() != mLinearity.Rows()) {
    mLinearityT.Init(mLinearity.Cols(), mLinearity.Rows());
    mShadowValid = false;
  }
  // the registry is keyed by W's address: an entry under an older address (W re-initialised with other
  // dimensions) would mirror the updates of whatever matrix is allocated there next into this layer's shadow
  DropShadowKey();
  TNET_SAFE_CALL(tnet_weight_shadow(mLinearity.pCUData(), mLinearity.Dim(), mLinearityT.pCUData(),
                                    (int)mLinearityT.Stride()));
  mShadowKey = mLinearity.pCUData();
  mShadowOn = true;
}

void CuBiasedLinearity::DropShadowKey() {
  if (mShadowKey && mShadowKey != mLinearity.pCUData()) {
    (void)tnet_weight_shadow(mShadowKey, TnetMatrixDim{}, nullptr, 0);
    mShadowValid = false;
  }
  mShadowKey = nullptr;
}

const CuMatrix<BaseFloat>& CuBiasedLinearity::ShadowForBwd() {
  if (!mShadowOn) Error("CuBiasedLinearity::ShadowForBwd: no shadow (UseShadow)");
  if (!mShadowValid) {
    KTScope kt("transpose:" + std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs()),
               8.0 * GetNInputs() * GetNOutputs());
    TNET_SAFE_CALL(tnet_transpose(mLinearity.pCUData(), mLinearity.Dim(), mLinearityT.pCUData(),
                                  (int)mLinearityT.Stride(), S));
    mShadowValid = true;
  }
  return mLinearityT;
}

void CuBiasedLinearity::BackpropUpdateRow(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                                          CuMatrix<BaseFloat>& Eout, const float* s, float* d) {
  CuProfileScope p("CuBiasedLinearity::BackpropUpdate");
  if (X.Rows() != 1 || E.Rows() != 1) Error("CuBiasedLinearity::BackpropUpdateRow: one frame only");
  float scale, l2;
  UpdateConstants(1, &scale, &l2);
  const bool mmt = mMomentum != 0.0f;
  Eout.Init(1, GetNInputs());
  TNET_SAFE_CALL(tnet_affine_bwd_update_row(X.pCUData(), (int)GetNInputs(), E.pCUData(), (int)GetNOutputs(),
                                            mLinearity.pCUData(), (int)mLinearity.Stride(),
                                            mmt ? mLinearityCorrection.pCUData() : nullptr,
                                            (int)mLinearityCorrection.Stride(), mBias.pCUData(),
                                            mmt ? mBiasCorrection.pCUData() : nullptr, scale, mMomentum, l2,
                                            Eout.pCUData(), s, d, S));
  mShadowValid = false;
}

void CuBiasedLinearity::UpdateFromColsum(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                                         const CuMatrix<BaseFloat>& colpart) {
  CuProfileScope p("CuBiasedLinearity::Update");
  float scale, l2;
  UpdateConstants(X.Rows(), &scale, &l2);
  const bool mmt = mMomentum != 0.0f;
  KTScope kt("gemm_upd:" + std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs()),
             2.0 * X.Rows() * GetNInputs() * GetNOutputs());
  TNET_SAFE_CALL(tnet_affine_update_bias(X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mLinearity.pCUData(),
                                         mLinearity.Dim(), mmt ? mLinearityCorrection.pCUData() : nullptr,
                                         (int)mLinearityCorrection.Stride(), scale, mMomentum, l2, colpart.pCUData(),
                                         (int)colpart.Stride(), mBias.pCUData(),
                                         mmt ? mBiasCorrection.pCUData() : nullptr, S));
  NoteUpdate();
}

bool CuBiasedLinearity::UpdateFromColsumWithBwd(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                                                const CuMatrix<BaseFloat>& colpart, const CuBiasedLinearity& below,
                                                const CuMatrix<BaseFloat>& E2, const CuMatrix<BaseFloat>& Ybelow,
                                                CuMatrix<BaseFloat>& Eo, CuMatrix<BaseFloat>& colpart2,
                                                bool use_shadow) {
  CuProfileScope p("CuBiasedLinearity::Update+Backpropagate");
  float scale, l2;
  UpdateConstants(X.Rows(), &scale, &l2);
  const bool mmt = mMomentum != 0.0f;
  const std::string su = std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs());
  const std::string sb = std::to_string(below.GetNInputs()) + "x" + std::to_string(below.GetNOutputs());
  KTScope kt("gemm_upd+bwd:" + (su == sb ? su : su + "+" + sb),
             2.0 * X.Rows() * GetNInputs() * GetNOutputs() + 2.0 * E2.Rows() * below.GetNInputs() * below.GetNOutputs(),
             2);
  // the lower layer's backward from its transposed shadow when it keeps one (NN, the forward's layout)
  // (the caller's decision, the same one its standalone backward takes: TrainBunch's `shadows`)
  const CuMatrix<BaseFloat>* wt =
      use_shadow && below.HasShadow() ? &const_cast<CuBiasedLinearity&>(below).ShadowForBwd() : nullptr;
  auto pair = wt ? tnet_affine_update_bwd_pair_t : tnet_affine_update_bwd_pair;
  const CuMatrix<BaseFloat>& wb = wt ? *wt : below.LinearityRO();
  const int st = pair(
      X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mLinearity.pCUData(), mLinearity.Dim(),
      mmt ? mLinearityCorrection.pCUData() : nullptr, (int)mLinearityCorrection.Stride(), scale, mMomentum, l2,
      colpart.pCUData(), (int)colpart.Stride(), mBias.pCUData(), mmt ? mBiasCorrection.pCUData() : nullptr,
      E2.pCUData(), E2.Dim(), wb.pCUData(), wb.Dim(), Ybelow.pCUData(),
      (int)Ybelow.Stride(), Eo.pCUData(), Eo.Dim(), colpart2.pCUData(), (int)colpart2.Stride(), S);
  if (st == TNET_ERR_UNSUPPORTED) {
    kt.Cancel();
    return false;
  }
  TNET_SAFE_CALL(st);
  NoteUpdate();
  return true;
}

bool CuBiasedLinearity::UpdatePairFromColsum(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                                             const CuMatrix<BaseFloat>& colpart, CuBiasedLinearity& other,
                                             const CuMatrix<BaseFloat>& X2, const CuMatrix<BaseFloat>& E2,
                                             const CuMatrix<BaseFloat>& colpart2) {
  CuProfileScope p("CuBiasedLinearity::Update (pair)");
  float scale, l2, scale2, l22;
  UpdateConstants(X.Rows(), &scale, &l2);
  other.UpdateConstants(X2.Rows(), &scale2, &l22);
  const bool mmt = mMomentum != 0.0f, mmt2 = other.mMomentum != 0.0f;
  const std::string sa = std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs());
  const std::string sb = std::to_string(other.GetNInputs()) + "x" + std::to_string(other.GetNOutputs());
  KTScope kt("gemm_upd+upd:" + sa + "+" + sb,
             2.0 * X.Rows() * GetNInputs() * GetNOutputs() + 2.0 * X2.Rows() * other.GetNInputs() * other.GetNOutputs(),
             2);
  const int st = tnet_affine_update_bias_pair(
      X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mLinearity.pCUData(), mLinearity.Dim(),
      mmt ? mLinearityCorrection.pCUData() : nullptr, (int)mLinearityCorrection.Stride(), scale, mMomentum, l2,
      colpart.pCUData(), (int)colpart.Stride(), mBias.pCUData(), mmt ? mBiasCorrection.pCUData() : nullptr,
      X2.pCUData(), X2.Dim(), E2.pCUData(), E2.Dim(), other.mLinearity.pCUData(), other.mLinearity.Dim(),
      mmt2 ? other.mLinearityCorrection.pCUData() : nullptr, (int)other.mLinearityCorrection.Stride(), scale2,
      other.mMomentum, l22, colpart2.pCUData(), (int)colpart2.Stride(), other.mBias.pCUData(),
      mmt2 ? other.mBiasCorrection.pCUData() : nullptr, S);
  if (st == TNET_ERR_UNSUPPORTED) {
    kt.Cancel();
    return false;
  }
  TNET_SAFE_CALL(st);
  NoteUpdate();
  other.NoteUpdate();
  return true;
}

bool CuBiasedLinearity::UpdateFromColsumGather(const CuMatrix<BaseFloat>& X, const CuMatrix<BaseFloat>& E,
                                               const CuMatrix<BaseFloat>& colpart, CuBiasedLinearity* other,
                                               const CuMatrix<BaseFloat>* X2, const CuMatrix<BaseFloat>* E2,
                                               const CuMatrix<BaseFloat>* colpart2, const BunchGather& g) {
  CuProfileScope p(other ? "CuBiasedLinearity::Update (pair) + gather" : "CuBiasedLinearity::Update + gather");
  float scale, l2, scale2 = 0.f, l22 = 0.f;
  UpdateConstants(X.Rows(), &scale, &l2);
  const bool mmt = mMomentum != 0.0f, mmt2 = other && other->mMomentum != 0.0f;
  if (other) other->UpdateConstants(X2->Rows(), &scale2, &l22);
  std::string name = "gemm_upd" + std::string(other ? "+upd" : "") + "+gather:" + std::to_string(GetNInputs()) + "x" +
                     std::to_string(GetNOutputs());
  double flops = 2.0 * X.Rows() * GetNInputs() * GetNOutputs();
  if (other) {
    name += "+" + std::to_string(other->GetNInputs()) + "x" + std::to_string(other->GetNOutputs());
    flops += 2.0 * X2->Rows() * other->GetNInputs() * other->GetNOutputs();
  }
  KTScope kt(name, flops, other ? 2 : 1);
  const TnetMatrixDim z{};
  const int st = tnet_affine_update_bias_gather(
      X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mLinearity.pCUData(), mLinearity.Dim(),
      mmt ? mLinearityCorrection.pCUData() : nullptr, (int)mLinearityCorrection.Stride(), scale, mMomentum, l2,
      colpart.pCUData(), (int)colpart.Stride(), mBias.pCUData(), mmt ? mBiasCorrection.pCUData() : nullptr,
      other ? X2->pCUData() : nullptr, other ? X2->Dim() : z, other ? E2->pCUData() : nullptr, other ? E2->Dim() : z,
      other ? other->mLinearity.pCUData() : nullptr, other ? other->mLinearity.Dim() : z,
      mmt2 ? other->mLinearityCorrection.pCUData() : nullptr, other ? (int)other->mLinearityCorrection.Stride() : 0,
      scale2, other ? other->mMomentum : 0.f, l22, other ? colpart2->pCUData() : nullptr,
      other ? (int)colpart2->Stride() : 0, other ? other->mBias.pCUData() : nullptr,
      mmt2 ? other->mBiasCorrection.pCUData() : nullptr, g.y, g.x, g.labels_out, g.labels_in, g.copy_from, g.dy, g.dx,
      S);
  if (st == TNET_ERR_UNSUPPORTED) {
    kt.Cancel();
    return false;
  }
  TNET_SAFE_CALL(st);
  NoteUpdate();
  if (other) other->NoteUpdate();
  return true;
}

void CuBiasedLinearity::Update() { UpdateFrom(GetInput(), GetErrorInput()); }

void CuBiasedLinearity::ComputeGradient() {
  CuProfileScope p("CuBiasedLinearity::ComputeGradient");
  const CuMatrix<BaseFloat>& X = GetInput();
  const CuMatrix<BaseFloat>& E = GetErrorInput();
  mGradW.Init(mLinearity.Rows(), mLinearity.Cols());
  mGradB.Init(mBias.Dim());
  KTScope kt("gemm_grad:" + std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs()),
             2.0 * X.Rows() * GetNInputs() * GetNOutputs());
  TNET_SAFE_CALL(tnet_affine_grad(X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mGradW.pCUData(), mGradW.Dim(), S));
  TnetMatrixDim dE = E.Dim();
  void* ws = CuDevice::Instantiate().Workspace((size_t)tnet_col_sum_workspace(dE));
  TNET_SAFE_CALL(tnet_bias_update(E.pCUData(), dE, nullptr, nullptr, mGradB.pCUData(), 0.f, 0.f, ws, S));
}

void CuBiasedLinearity::ComputeGradientColsum(const CuMatrix<BaseFloat>& colpart) {
  CuProfileScope p("CuBiasedLinearity::ComputeGradient");
  const CuMatrix<BaseFloat>& X = GetInput();
  const CuMatrix<BaseFloat>& E = GetErrorInput();
  mGradW.Init(mLinearity.Rows(), mLinearity.Cols());
  mGradB.Init(mBias.Dim());
  KTScope kt("gemm_grad:" + std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs()),
             2.0 * X.Rows() * GetNInputs() * GetNOutputs());
  TNET_SAFE_CALL(tnet_affine_grad_bias(X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mGradW.pCUData(), mGradW.Dim(),
                                       colpart.pCUData(), (int)colpart.Stride(), mGradB.pCUData(), S));
}

bool CuBiasedLinearity::ComputeGradientColsumGather(const CuMatrix<BaseFloat>& colpart, const BunchGather& g,
                                                    CuBiasedLinearity* other, const CuMatrix<BaseFloat>* colpart2) {
  CuProfileScope p(other ? "CuBiasedLinearity::ComputeGradient (pair) + gather" : "CuBiasedLinearity::ComputeGradient + gather");
  const CuMatrix<BaseFloat>& X = GetInput();
  const CuMatrix<BaseFloat>& E = GetErrorInput();
  mGradW.Init(mLinearity.Rows(), mLinearity.Cols());
  mGradB.Init(mBias.Dim());
  std::string name = "gemm_grad" + std::string(other ? "+grad" : "") + "+gather:" + std::to_string(GetNInputs()) + "x" +
                     std::to_string(GetNOutputs());
  double flops = 2.0 * X.Rows() * GetNInputs() * GetNOutputs();
  const TnetMatrixDim z{};
  const float* X2 = nullptr;
  const float* E2 = nullptr;
  TnetMatrixDim dX2 = z, dE2 = z, dG2 = z;
  if (other) {
    other->mGradW.Init(other->mLinearity.Rows(), other->mLinearity.Cols());
    other->mGradB.Init(other->mBias.Dim());
    X2 = other->GetInput().pCUData();
    dX2 = other->GetInput().Dim();
    E2 = other->GetErrorInput().pCUData();
    dE2 = other->GetErrorInput().Dim();
    dG2 = other->mGradW.Dim();
    name += "+" + std::to_string(other->GetNInputs()) + "x" + std::to_string(other->GetNOutputs());
    flops += 2.0 * other->GetInput().Rows() * other->GetNInputs() * other->GetNOutputs();
  }
  KTScope kt(name, flops, other ? 2 : 1);
  const int st = tnet_affine_grad_bias_gather(
      X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mGradW.pCUData(), mGradW.Dim(), colpart.pCUData(),
      (int)colpart.Stride(), mGradB.pCUData(), X2, dX2, E2, dE2, other ? other->mGradW.pCUData() : nullptr, dG2,
      other ? colpart2->pCUData() : nullptr, other ? (int)colpart2->Stride() : 0,
      other ? other->mGradB.pCUData() : nullptr, g.y, g.x, g.labels_out, g.labels_in, g.copy_from, g.dy, g.dx, S);
  if (st == TNET_ERR_UNSUPPORTED) {
    kt.Cancel();
    return false;
  }
  TNET_SAFE_CALL(st);
  return true;
}

bool CuBiasedLinearity::ComputeGradientColsumWithBwd(const CuMatrix<BaseFloat>& colpart, const CuBiasedLinearity& below,
                                                     const CuMatrix<BaseFloat>& E2, const CuMatrix<BaseFloat>& Ybelow,
                                                     CuMatrix<BaseFloat>& Eo, CuMatrix<BaseFloat>& colpart2) {
  CuProfileScope p("CuBiasedLinearity::ComputeGradient+Backpropagate");
  const CuMatrix<BaseFloat>& X = GetInput();
  const CuMatrix<BaseFloat>& E = GetErrorInput();
  mGradW.Init(mLinearity.Rows(), mLinearity.Cols());
  mGradB.Init(mBias.Dim());
  const std::string su = std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs());
  const std::string sb = std::to_string(below.GetNInputs()) + "x" + std::to_string(below.GetNOutputs());
  KTScope kt("gemm_grad+bwd:" + (su == sb ? su : su + "+" + sb),
             2.0 * X.Rows() * GetNInputs() * GetNOutputs() + 2.0 * E2.Rows() * below.GetNInputs() * below.GetNOutputs(),
             2);
  const int st = tnet_affine_grad_bwd_pair(
      X.pCUData(), X.Dim(), E.pCUData(), E.Dim(), mGradW.pCUData(), mGradW.Dim(), colpart.pCUData(),
      (int)colpart.Stride(), mGradB.pCUData(), E2.pCUData(), E2.Dim(), below.Linearity().pCUData(),
      below.Linearity().Dim(), Ybelow.pCUData(), (int)Ybelow.Stride(), Eo.pCUData(), Eo.Dim(), colpart2.pCUData(),
      (int)colpart2.Stride(), S);
  if (st == TNET_ERR_UNSUPPORTED) {
    kt.Cancel();
    return false;
  }
  TNET_SAFE_CALL(st);
  return true;
}

std::vector<CuParamBlock> CuBiasedLinearity::GradientBlocks() {
  mGradW.Init(mLinearity.Rows(), mLinearity.Cols());
  mGradB.Init(mBias.Dim());
  return {CuParamBlock{mGradW.pCUData(), (long)(mGradW.Rows() * mGradW.Stride()), mLinearity.pCUData()},
          CuParamBlock{mGradB.pCUData(), (long)mGradB.Dim(), mBias.pCUData()}};
}

int CuBiasedLinearity::ApplySegments(size_t frames, const GradExchange* ex, TnetSgdSeg* seg, float* scale) {
  float l2;
  UpdateConstants(frames, scale, &l2);
  const bool mmt = mMomentum != 0.0f;
  mShadowValid = false;  // the flat apply writes no transposed shadow
  // padding columns of W and of the gradient are zero, so the flat update keeps them zero; W and b
  // in one launch, each as the element ranges this rank applies (sharded apply: its shard + the tail)
  int nseg = 0;
  auto add = [&](float* prm, float* grd, float* corr, long n, float wl2) {
    long lo[2], hi[2];
    const int nr = ex ? ex->ApplyRanges(n, lo, hi) : GradExchange::FullRange(n, lo, hi);
    for (int k = 0; k < nr; ++k)
      if (hi[k] > lo[k]) seg[nseg++] = {prm + lo[k], grd + lo[k], corr ? corr + lo[k] : nullptr, hi[k] - lo[k], wl2};
  };
  add(mLinearity.pCUData(), mGradW.pCUData(), mmt ? mLinearityCorrection.pCUData() : nullptr,
      (long)(mLinearity.Rows() * mLinearity.Stride()), l2);
  add(mBias.pCUData(), mGradB.pCUData(), mmt ? mBiasCorrection.pCUData() : nullptr, (long)mBias.Dim(), 0.f);
  return nseg;
}

void CuBiasedLinearity::ApplyGradient(size_t frames, void* stream, const GradExchange* ex) {
  CuProfileScope p("CuBiasedLinearity::ApplyGradient");
  TnetSgdSeg seg[4];
  float scale;
  const int nseg = ApplySegments(frames, ex, seg, &scale);
  if (stream) {  // beside the compute stream (GradExchange::ApplyStream): no library-stream timing
    TNET_SAFE_CALL(tnet_sgd_update_multi(seg, nseg, scale, mMomentum, stream));
    return;
  }
  KTScope kt("sgd_apply:" + std::to_string(GetNInputs()) + "x" + std::to_string(GetNOutputs()),
             12.0 * (double)(mLinearity.Rows() * mLinearity.Stride() + mBias.Dim()));
  TNET_SAFE_CALL(tnet_sgd_update_multi(seg, nseg, scale, mMomentum, S));
}

void CuBiasedLinearity::ApplyGradients(CuBiasedLinearity* const* ls, int n, size_t frames, const GradExchange* ex) {
  CuProfileScope p("CuBiasedLinearity::ApplyGradient");
  TnetSgdSeg seg[8];
  float scale[2];
  bool same = n == 2 && ls[0]->mMomentum == ls[1]->mMomentum;
  int nseg = 0;
  for (int i = 0; i < n && same; ++i) nseg += ls[i]->ApplySegments(frames, ex, seg + nseg, &scale[i]);
  if (!same || scale[0] != scale[1]) {  // other constants: one launch per layer
    for (int i = 0; i < n; ++i) ls[i]->ApplyGradient(frames, nullptr, ex);
    return;
  }
  double bytes = 0.0;
  for (int i = 0; i < nseg; ++i) bytes += 12.0 * (double)seg[i].n;
  KTScope kt("sgd_apply:" + std::to_string(n) + "layers", bytes);
  TNET_SAFE_CALL(tnet_sgd_update_multi(seg, nseg, scale[0], ls[0]->mMomentum, S));
}

void CuBiasedLinearity::ReadFromStream(std::istream& rIn) {
  // matrix is stored transposed as SNet does (cuBiasedLinearity.cc:70-102)
  BfMatrix transpose;
  ReadMatrixFast(rIn, transpose);
  BfVector bias;
  ReadVectorFast(rIn, bias);
  if (transpose.Cols() * transpose.Rows() == 0) Error("Missing linearity matrix in network file");
  if (bias.Dim() == 0) Error("Missing bias vector in network file");
  if (transpose.Rows() != GetNOutputs() || transpose.Cols() != GetNInputs() || bias.Dim() != GetNOutputs()) {
    std::ostringstream os;
    os << "Wrong dimensionalities of matrix/vector in network file\n"
       << "Inputs:" << GetNInputs() << "Outputs:" << GetNOutputs() << "\n"
       << "linearityCols:" << transpose.Rows() << "linearityRows:" << transpose.Cols() << "biasDims:" << bias.Dim()
       << "\n";
    Error(os.str());
  }
  mLinearity.CopyFrom(BfMatrix(transpose, TRANS));
  mBias.CopyFrom(bias);
  mShadowValid = false;
  if (mShadowOn) UseShadow();  // W's storage may have moved: re-key the registration
}

void CuBiasedLinearity::WriteToStream(std::ostream& rOut) {
  BfMatrix tmp;
  mLinearity.CopyTo(tmp);
  BfMatrix transpose(tmp, TRANS);
  rOut << transpose;
  BfVector vec;
  mBias.CopyTo(vec);
  rOut << vec;
  rOut << std::endl;
}

// ----------------------------------------------------------------------- activations
void CuSigmoid::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) { CuMath<BaseFloat>::Sigmoid(Y, X); }
void CuSigmoid::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  CuMath<BaseFloat>::DiffSigmoid(Y, X, mOutput);
}
void CuSoftmax::PropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) { CuMath<BaseFloat>::Softmax(Y, X); }
void CuSoftmax::BackpropagateFnc(const CuMatrix<BaseFloat>& X, CuMatrix<BaseFloat>& Y) {
  // we assume X is already dE/dSoftmax_input (cuActivation.cc:37-40)
  Y.CopyFrom(X);
}

}  // namespace TNet
