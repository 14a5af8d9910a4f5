// cunetwork.cpp -- see cunetwork.h.
#include "cunetwork.h"

#include "cufeat.h"
#include "curbm.h"
#include "curecurrent.h"

#include <algorithm>
#include <cctype>
#include <fstream>
#include <list>

#include "gradexchange.h"

namespace TNet {

#define S ((void*)CuDevice::Instantiate().Stream())

CuNetwork::~CuNetwork() {
  for (auto*& c : mNetComponents) {
    delete c;
    c = nullptr;
  }
}

void CuNetwork::AddLayer(CuComponent* layer) {
  if (!mNetComponents.empty()) {
    if (GetNOutputs() != layer->GetNInputs()) Error("Nonmatching dims");
    layer->SetInput(mNetComponents.back()->GetOutput());
    mNetComponents.back()->SetErrorInput(layer->GetErrorOutput());
  }
  mNetComponents.push_back(layer);
}

size_t CuNetwork::GetNInputs() const { return mNetComponents.empty() ? 0 : mNetComponents.front()->GetNInputs(); }
size_t CuNetwork::GetNOutputs() const { return mNetComponents.empty() ? 0 : mNetComponents.back()->GetNOutputs(); }

void CuNetwork::Propagate(const CuMatrix<BaseFloat>& in, CuMatrix<BaseFloat>& out) {
  if (mNetComponents.empty()) {
    out.CopyFrom(in);
    return;
  }
  if (in.Cols() != GetNInputs()) {
    std::ostringstream os;
    os << "Nonmatching dims data dim is: " << in.Cols() << " network needs: " << GetNInputs();
    Error(os.str());
  }
  mNetComponents.front()->SetInput(in);
  for (auto* c : mNetComponents) c->Propagate();
  out.CopyFrom(mNetComponents.back()->GetOutput());
}

void CuNetwork::Backpropagate(const CuMatrix<BaseFloat>& globerr) {
  mNetComponents.back()->SetErrorInput(globerr);
  for (auto it = mNetComponents.rbegin(); it != mNetComponents.rend(); ++it) {
    if (*it != mpPropagErrorStopper) (*it)->Backpropagate();
    if ((*it)->IsUpdatable()) {
      CuUpdatableComponent& rComp = dynamic_cast<CuUpdatableComponent&>(**it);
      if (rComp.LearnRate() > 0.0f) rComp.Update();
    }
    if (mpPropagErrorStopper == *it) break;
  }
}

void CuNetwork::ReadNetwork(const char* pSrc) {
  std::ifstream in(pSrc);
  if (!in.good()) Error(std::string("Error, cannot read model: ") + pSrc);
  ReadNetwork(in);
}

void CuNetwork::WriteNetwork(const char* pDst) {
  std::ofstream out(pDst);
  if (!out.good()) Error(std::string("Error, cannot write model: ") + pDst);
  WriteNetwork(out);
}

void CuNetwork::ReadNetwork(std::istream& rIn) {
  CuComponent* pComp;
  while (nullptr != (pComp = ComponentFactory(rIn))) mNetComponents.push_back(pComp);
}

void CuNetwork::WriteNetwork(std::ostream& rOut) {
  for (auto* c : mNetComponents) ComponentDumper(rOut, *c);
}

void CuNetwork::SetLearnRate(BaseFloat learnRate, const char* pLearnRateFactors) {
  // cuNetwork.cc:80-134
  std::list<BaseFloat> lr_factors;
  if (pLearnRateFactors) {
    std::string str(pLearnRateFactors);
    for (auto& ch : str)
      if (ch == ':' || ch == ',') ch = ' ';
    std::istringstream is(str);
    BaseFloat f;
    while (is >> f) lr_factors.push_back(f);
    mLearnRateFactors = pLearnRateFactors;
  }
  BaseFloat scale = 1.0f;
  mGlobLearnRate = learnRate;
  bool stopper_given = false;
  mpPropagErrorStopper = nullptr;
  for (auto* c : mNetComponents) {
    if (c->IsUpdatable()) {
      if (pLearnRateFactors) {
        if (lr_factors.empty()) Error("Too few learninig rate scale factors");
        scale = lr_factors.front();
        lr_factors.pop_front();
      }
      dynamic_cast<CuUpdatableComponent*>(c)->LearnRate(learnRate * scale);
      if (!stopper_given && (learnRate * scale > 0.0)) {
        mpPropagErrorStopper = c;
        stopper_given = true;
      }
    }
  }
  if (!lr_factors.empty()) Error("Too much learninig rate scale factors");
}

void CuNetwork::PrintLearnRate() {
  std::cout << "Learning rate: global " << mGlobLearnRate << " components' ";
  for (auto* c : mNetComponents)
    if (c->IsUpdatable()) std::cout << " " << dynamic_cast<CuUpdatableComponent*>(c)->LearnRate();
  std::cout << "\n" << std::flush;
}

void CuNetwork::SetMomentum(BaseFloat momentum) {
  for (auto* c : mNetComponents)
    if (c->IsUpdatable()) dynamic_cast<CuUpdatableComponent*>(c)->Momentum(momentum);
}
void CuNetwork::SetWeightcost(BaseFloat weightcost) {
  for (auto* c : mNetComponents)
    if (c->IsUpdatable()) dynamic_cast<CuUpdatableComponent*>(c)->Weightcost(weightcost);
}
void CuNetwork::SetL1(BaseFloat l1) {
  // only <sparselinearity> uses L1 (cuNetwork.cc:159-168); not part of this build's component set
  (void)l1;
}
void CuNetwork::SetGradDivFrm(bool div) {
  for (auto* c : mNetComponents)
    if (c->IsUpdatable()) dynamic_cast<CuUpdatableComponent*>(c)->GradDivFrm(div);
}

CuComponent* CuNetwork::ComponentFactory(std::istream& rIn) {
  rIn >> std::ws;
  if (rIn.eof()) return nullptr;
  std::string tag;
  rIn >> tag;
  if (tag.empty()) return nullptr;
  std::transform(tag.begin(), tag.end(), tag.begin(), ::tolower);
  if (tag[0] != '<' || tag[tag.size() - 1] != '>') Error(std::string("Invalid component tag:") + tag);
  if (tag == "<endblock>") return nullptr;
  size_t nInputs = 0, nOutputs = 0;
  rIn >> std::ws >> nOutputs >> std::ws >> nInputs;
  if (rIn.fail() || nInputs == 0 || nOutputs == 0) Error("Invalid component dimensions for " + tag);
  CuComponent* pPred = mNetComponents.empty() ? nullptr : mNetComponents.back();
  CuComponent* pRet = nullptr;
  if (tag == "<biasedlinearity>") pRet = new CuBiasedLinearity(nInputs, nOutputs, pPred);
  else if (tag == "<sigmoid>") pRet = new CuSigmoid(nInputs, nOutputs, pPred);
  else if (tag == "<softmax>") pRet = new CuSoftmax(nInputs, nOutputs, pPred);
  else if (tag == "<rbm>") pRet = new CuRbm(nInputs, nOutputs, pPred);
  else if (tag == "<recurrent>") pRet = new CuRecurrent(nInputs, nOutputs, pPred);
  // feature front end (cuNetwork.cc:263-268, cuCRBEDctFeat.h)
  else if (tag == "<expand>") pRet = new CuExpand(nInputs, nOutputs, pPred);
  else if (tag == "<copy>") pRet = new CuCopy(nInputs, nOutputs, pPred);
  else if (tag == "<transpose>") pRet = new CuTranspose(nInputs, nOutputs, pPred);
  else if (tag == "<blocklinearity>") pRet = new CuBlockLinearity(nInputs, nOutputs, pPred);
  else if (tag == "<bias>") pRet = new CuBias(nInputs, nOutputs, pPred);
  else if (tag == "<window>") pRet = new CuWindow(nInputs, nOutputs, pPred);
  else if (tag == "<log>") pRet = new CuLog(nInputs, nOutputs, pPred);
  else Error(std::string("Unknown Component tag:") + tag);
  pRet->ReadFromStream(rIn);
  return pRet;
}

void CuNetwork::ComponentDumper(std::ostream& rOut, CuComponent& rComp) {
  rOut << rComp.GetName() << " " << rComp.GetNOutputs() << " " << rComp.GetNInputs() << std::endl;
  rComp.WriteToStream(rOut);
}

// ======================================================================================
// fused training step
// ======================================================================================
bool CuNetwork::IsFusableMLP() const {
  const size_t n = mNetComponents.size();
  if (n < 2 || n % 2) return false;
  for (size_t i = 0; i < n; i += 2) {
    if (mNetComponents[i]->GetType() != CuComponent::BIASED_LINEARITY) return false;
    const bool last = (i + 2 == n);
    const CuComponent::ComponentType want = last ? CuComponent::SOFTMAX : CuComponent::SIGMOID;
    if (mNetComponents[i + 1]->GetType() != want) return false;
  }
  return true;
}

void CuNetwork::TrainBunchGeneric(const CuMatrix<BaseFloat>& X, const CuVector<int>& labels,
                                  CuObjectiveFunction& obj, bool train) {
  CuMatrix<BaseFloat> out;
  Propagate(X, out);
  obj.EvaluateLabels(out, labels, mGlobErr);
  if (train) Backpropagate(mGlobErr);
}

void CuNetwork::TrainEmpty(GradExchange& exchange) {
  if (!IsFusableMLP()) Error("CuNetwork::TrainEmpty: data-parallel training needs the sigmoid-MLP topology");
  const int nl = (int)mNetComponents.size() / 2;
  const size_t grows = exchange.GlobalRows(0);
  // the collectives in TrainBunch's order (top down to the stopper; a layer's reduction, then -- with
  // an apply stream -- its apply and parameter gather before the next layer's reduction), so every
  // rank issues the same sequence whether it trained a bunch or not
  std::vector<CuBiasedLinearity*> submitted;
  int n_submitted = 0;
  for (int l = nl - 1; l >= 0; l--) {
    auto* lin = static_cast<CuBiasedLinearity*>(mNetComponents[2 * l]);
    if (lin->LearnRate() > 0.0f) {
      lin->ZeroGradient();
      exchange.Submit(*lin);
      void* as = submitted.empty() ? exchange.ApplyStream(n_submitted) : nullptr;
      if (as) {
        lin->ApplyGradient(grows, as, &exchange);
        exchange.GatherParams(*lin, n_submitted, as);
      } else {
        submitted.push_back(lin);
      }
      n_submitted++;
    }
    if (lin == mpPropagErrorStopper) break;
  }
  const int first = n_submitted - (int)submitted.size();
  for (size_t i = 0; i < submitted.size(); i++) {
    exchange.WaitFor(first + (int)i);
    submitted[i]->ApplyGradient(grows, nullptr, &exchange);
    exchange.GatherParams(*submitted[i], first + (int)i, nullptr);
  }
  exchange.WaitAll();
}

void CuUpdatableComponent::ZeroGradient() {
  for (auto& b : GradientBlocks())
    TNET_HIP_CALL(hipMemsetAsync(b.grad, 0, (size_t)b.n * sizeof(float), CuDevice::Instantiate().Stream()));
}

// fault injection (tnet_debug_fail_train_bunch): the n-th next TrainBunch throws before it enqueues anything
static long g_fail_train_bunch = 0;
void CuNetwork::DebugFailTrainBunch(long n) { g_fail_train_bunch = n; }

// TNET_DP_PAIR=0: the data-parallel step never pairs a gradient GEMM with the backward GEMM below (A/B)
static const bool g_dp_pair = !(getenv("TNET_DP_PAIR") && getenv("TNET_DP_PAIR")[0] == '0');

void CuNetwork::TrainBunch(const CuMatrix<BaseFloat>& X, const CuVector<int>& labels, CuObjectiveFunction& obj,
                           bool train, GradExchange* exchange) {
  if (g_fail_train_bunch > 0 && --g_fail_train_bunch == 0) Error("CuNetwork::TrainBunch: injected fault");
  if (!IsFusableMLP() || obj.GetTypeId() != CuObjectiveFunction::CROSS_ENTROPY) {
    if (exchange) Error("CuNetwork::TrainBunch: data-parallel training needs the sigmoid-MLP topology");
    TrainBunchGeneric(X, labels, obj, train);
    return;
  }
  if (X.Cols() != GetNInputs()) Error("CuNetwork::TrainBunch: non-matching input dim");
  if (labels.Dim() != X.Rows()) Error("CuNetwork::TrainBunch: number of labels != rows");
  const size_t rows = X.Rows();
  const int nl = (int)mNetComponents.size() / 2;
  if (mErr.size() != (size_t)nl) {
    mErr.clear();
    mColPart.clear();
    for (int l = 0; l < nl; l++) {
      mErr.emplace_back(new CuMatrix<BaseFloat>());
      mColPart.emplace_back(new CuMatrix<BaseFloat>());
    }
  }
  mNetComponents.front()->SetInput(X);
  // the backward GEMMs read each weight's transposed shadow (NN: the forward's layout and direct form), which the
  // fused updates keep current in the same pass (CuBiasedLinearity::UseShadow; not in the data-parallel step, whose
  // flat SGD apply writes no shadow).  TNET_BWD_SHADOW: 2 (default) the hidden layers' backward GEMMs, whose 2048^2
  // shadow costs the update ~1 us and saves the backward ~5 (the top layer's 32 MB shadow costs its update 12 us for
  // an 8.5 us faster backward: profiles/r05_bwd_shadow_ab.json); 1 every layer above the first; 0 none (NT from W)
  static const int use_shadow = getenv("TNET_BWD_SHADOW") ? atoi(getenv("TNET_BWD_SHADOW")) : 2;
  const bool shadows = use_shadow > 0 && train && !exchange;
  if (shadows)
    for (int l = 1; l < (use_shadow == 2 ? nl - 1 : nl); l++)
      static_cast<CuBiasedLinearity*>(mNetComponents[2 * l])->UseShadow();

  // objective outputs: the error (+ the softmax output when kept)
  CuComponent* smx = mNetComponents.back();
  float* yout = nullptr;
  int ystride = 0;
  if (mKeepOutput) {
    smx->Output().Init(rows, smx->GetNOutputs());
    yout = smx->Output().pCUData();
    ystride = (int)smx->Output().Stride();
  }
  mGlobErr.Init(rows, GetNOutputs());
  // the top layer's bias gradient as slab sums (the update GEMM applies it)
  auto* top = static_cast<CuBiasedLinearity*>(mNetComponents[2 * (nl - 1)]);
  const bool top_colsum = train && top->LearnRate() > 0.0f;
  bool err_colsum = false;

  // ---- forward: act_{l+1} = sigmoid(act_l W_l + b_l) straight into the <sigmoid>'s output
  const CuMatrix<BaseFloat>* act = &X;
  std::vector<const CuMatrix<BaseFloat>*> acts(nl + 1);
  acts[0] = &X;
  bool fused_top = false;
  for (int l = 0; l < nl; l++) {
    auto* lin = static_cast<CuBiasedLinearity*>(mNetComponents[2 * l]);
    CuComponent* actc = mNetComponents[2 * l + 1];
    const bool last = (l == nl - 1);
    CuMatrix<BaseFloat>& dst = last ? lin->Output() : actc->Output();
    dst.Init(rows, lin->GetNOutputs());
    const std::string shape = std::to_string(lin->GetNInputs()) + "x" + std::to_string(lin->GetNOutputs());
    // TNET_FUSED_TOP=0: the three-call form (A/B measurements)
    static const bool fuse_top = !(getenv("TNET_FUSED_TOP") && getenv("TNET_FUSED_TOP")[0] == '0');
    if (last && fuse_top && lin->GetNOutputs() <= TNET_AFFINE_SOFTMAX_MAX_N) {
      // up to 256 classes: logits, softmax, xent, error and the error's slab sums in one pass
      float* cp = nullptr;
      int ldcp = 0;
      if (top_colsum) {
        mColPart[l]->Init(tnet_colsum_slabs((int)rows), lin->GetNOutputs());
        cp = mColPart[l]->pCUData();
        ldcp = (int)mColPart[l]->Stride();
      }
      KTScope kt("gemm_fwd+softmax:" + shape, 2.0 * rows * lin->GetNInputs() * lin->GetNOutputs());
      const int st = tnet_affine_softmax_xent(act->pCUData(), act->Dim(), lin->LinearityRO().pCUData(),
                                              lin->LinearityRO().Dim(), lin->Bias().pCUData(), labels.pCUData(),
                                              dst.pCUData(), (int)dst.Stride(), yout, ystride, mGlobErr.pCUData(),
                                              (int)mGlobErr.Stride(), obj.DeviceStats(), cp, ldcp, S);
      if (st != TNET_ERR_UNSUPPORTED) {
        TNET_SAFE_CALL(st);
        fused_top = true;
        err_colsum = top_colsum;
        acts[l + 1] = &dst;
        break;
      }
    }
    KTScope kt("gemm_fwd:" + shape, 2.0 * rows * lin->GetNInputs() * lin->GetNOutputs());
    TNET_SAFE_CALL(tnet_affine_fwd(act->pCUData(), act->Dim(), lin->LinearityRO().pCUData(), lin->LinearityRO().Dim(),
                                   lin->Bias().pCUData(), dst.pCUData(), dst.Dim(), last ? 0 : 1, S));
    act = &dst;
    acts[l + 1] = &dst;
  }
  // ---- objective: softmax + xent + error (+ optional softmax output); the error's slab sums (the top layer's bias
  // gradient) ride on the top layer's backward launch below.  (Round 2's one-pass softmax + slab sums,
  // tnet_softmax_xent_slabs, was measured slower -- 36.7 us against 9.8 + 6.7 us, profiles/r02_softmax_slabs_ab.txt
  // -- and is gone since round 6.)
  if (!fused_top) {
    CuMatrix<BaseFloat>& logits = mNetComponents[2 * (nl - 1)]->Output();
    KTScope kts("softmax_xent:" + std::to_string(GetNOutputs()),
                (double)rows * GetNOutputs() * 4.0 * (mKeepOutput ? 3 : 2) + rows * 4.0);
    TNET_SAFE_CALL(tnet_softmax_xent(logits.pCUData(), logits.Dim(), labels.pCUData(), yout, ystride, mGlobErr.pCUData(),
                                     (int)mGlobErr.Stride(), obj.DeviceStats(), S));
  }
  obj.AddFrames(rows);
  if (!train) return;

  // ---- backward + update, top to bottom (error uses the pre-update weights of the layer)
  const CuMatrix<BaseFloat>* err = &mGlobErr;
  std::vector<CuBiasedLinearity*> submitted;  // data-parallel: layers in reduction order, not yet applied
  const size_t grows = exchange ? exchange->GlobalRows(rows) : rows;
  int n_submitted = 0;
  // the top layer's bias gradient (the softmax error's slab sums): carried by the top layer's backward launch
  // where that launch takes it (tnet_affine_bwd_colsum_slabs, its blocks on the CUs the GEMM tiles free;
  // TNET_TOP_SLABS_RIDE=0: a launch of its own here)
  static const bool slabs_ride = !(getenv("TNET_TOP_SLABS_RIDE") && getenv("TNET_TOP_SLABS_RIDE")[0] == '0');
  bool top_slabs_ride = false;
  auto top_slabs_launch = [&]() {
    CuMatrix<BaseFloat>& cp = *mColPart[nl - 1];
    KTScope kt("colsum:" + std::to_string(GetNOutputs()), 4.0 * rows * GetNOutputs());
    const int st = tnet_colsum_slab_sums(mGlobErr.pCUData(), mGlobErr.Dim(), cp.pCUData(), (int)cp.Stride(), S);
    if (st == TNET_ERR_UNSUPPORTED) return false;
    TNET_SAFE_CALL(st);
    return true;
  };
  if (top_colsum && !fused_top && !err_colsum) {
    mColPart[nl - 1]->Init(tnet_colsum_slabs((int)rows), GetNOutputs());
    const bool top_bwd = nl > 1 && mNetComponents[2 * (nl - 1)] != mpPropagErrorStopper &&
                         static_cast<CuBiasedLinearity*>(mNetComponents[2 * (nl - 2)])->LearnRate() > 0.0f;
    if (slabs_ride && top_bwd) top_slabs_ride = err_colsum = true;  // settled by the top layer's backward below
    else err_colsum = top_slabs_launch();
  }  // slab column sums of *err are in mColPart[l] (bias gradient fused, no exchange)
  // Without data parallelism the fused update of layer l is held back one layer and enqueued with the
  // backward GEMM of layer l-1 as ONE launch where the pair kernel takes both shapes
  // (tnet_affine_update_bwd_pair: the two are independent -- layer l-1's backward reads W_{l-1} only);
  // otherwise (or TNET_GEMM_PAIR=0 in the library) the update runs right before that backward GEMM.
  struct Pending {
    CuBiasedLinearity* lin = nullptr;
    const CuMatrix<BaseFloat>* X = nullptr;
    const CuMatrix<BaseFloat>* E = nullptr;
    int l = -1;
  } pend;
  auto flush = [&]() {
    if (!pend.lin) return;
    pend.lin->UpdateFromColsum(*pend.X, *pend.E, *mColPart[pend.l]);
    pend.lin = nullptr;
  };
  // Data parallel: a layer's reduction submitted, and its SGD apply right behind it (beside the backward GEMMs
  // below: W_l is read for the last time by this layer's backward GEMM, already enqueued) -- the step's last layer
  // on the compute stream (nothing is left to overlap it with, and the apply stream would add a hop in and a join
  // out; TNET_DP_LAST_APPLY_STREAM=1: on the apply stream too, A/B)
  static const bool last_on_apply = getenv("TNET_DP_LAST_APPLY_STREAM") && getenv("TNET_DP_LAST_APPLY_STREAM")[0] == '1';
  auto submit_layer = [&](CuBiasedLinearity* lin, bool last) {
    exchange->Submit(*lin);
    void* as = submitted.empty() && (!last || last_on_apply) ? exchange->ApplyStream(n_submitted) : nullptr;
    if (as) {
      lin->ApplyGradient(grows, as, exchange);
      exchange->GatherParams(*lin, n_submitted, as);  // sharded apply: the other ranks' shards
    } else {
      submitted.push_back(lin);
    }
    n_submitted++;
  };
  // ... and, while no CUs are reserved for RCCL (tnet_gemm_reserve: before the step's first submission, or a
  // single-rank communicator), a layer's gradient GEMM is held back one layer and enqueued with the backward GEMM
  // of the layer below as ONE launch (tnet_affine_grad_bwd_pair, the pair kernel of the fused step; independent:
  // the gradient reads X_l, E_l, the backward E_l and W_{l-1})
  CuBiasedLinearity* pgrad = nullptr;
  int pgrad_l = -1;
  auto flush_grad = [&]() {
    if (!pgrad) return;
    pgrad->ComputeGradientColsum(*mColPart[pgrad_l]);
    submit_layer(pgrad, false);
    pgrad = nullptr;
  };
  for (int l = nl - 1; l >= 0; l--) {
    auto* lin = static_cast<CuBiasedLinearity*>(mNetComponents[2 * l]);
    const bool stopper = (lin == mpPropagErrorStopper);
    CuMatrix<BaseFloat>* eo = nullptr;
    bool eo_colsum = false;
    if (!stopper && l > 0) {
      eo = mErr[l].get();
      eo->Init(rows, lin->GetNInputs());
      const std::string shape = std::to_string(lin->GetNInputs()) + "x" + std::to_string(lin->GetNOutputs());
      // E_l = (E_{l+1} W_l^T) .* y_l (1 - y_l)   (backprop through <biasedlinearity> and the <sigmoid> below);
      // when the layer below is trained here, the same launch writes the bias gradient of E_l as slab sums
      auto* below = static_cast<CuBiasedLinearity*>(mNetComponents[2 * (l - 1)]);
      if (below->LearnRate() > 0.0f) {
        CuMatrix<BaseFloat>& cp = *mColPart[l - 1];
        cp.Init(tnet_colsum_slabs((int)rows), lin->GetNInputs());
        if (pgrad && pgrad->ComputeGradientColsumWithBwd(*mColPart[pgrad_l], *lin, *err, *acts[l], *eo, cp)) {
          submit_layer(pgrad, false);
          pgrad = nullptr;
          eo_colsum = true;
        } else if (pend.lin && pend.lin->UpdateFromColsumWithBwd(*pend.X, *pend.E, *mColPart[pend.l], *lin, *err,
                                                                *acts[l], *eo, cp, shadows)) {
          pend.lin = nullptr;
          eo_colsum = true;
        } else {
          flush_grad();
          flush();
          KTScope kt("gemm_bwd:" + shape, 2.0 * rows * lin->GetNInputs() * lin->GetNOutputs());
          int st = TNET_ERR_UNSUPPORTED;
          if (top_slabs_ride) {  // l == nl - 1: err is the softmax error
            top_slabs_ride = false;
            CuMatrix<BaseFloat>& ct = *mColPart[nl - 1];
            const bool t = shadows && lin->HasShadow();
            const CuMatrix<BaseFloat>& wb = t ? lin->ShadowForBwd() : lin->LinearityRO();
            st = (t ? tnet_affine_bwd_colsum_slabs_t : tnet_affine_bwd_colsum_slabs)(
                err->pCUData(), err->Dim(), wb.pCUData(), wb.Dim(), acts[l]->pCUData(), (int)acts[l]->Stride(),
                eo->pCUData(), eo->Dim(), cp.pCUData(), (int)cp.Stride(), ct.pCUData(), (int)ct.Stride(), S);
            if (st == TNET_ERR_UNSUPPORTED) err_colsum = top_slabs_launch();
          }
          if (st == TNET_ERR_UNSUPPORTED && shadows && lin->HasShadow()) {
            const CuMatrix<BaseFloat>& wt = lin->ShadowForBwd();
            st = tnet_affine_bwd_colsum_t(err->pCUData(), err->Dim(), wt.pCUData(), wt.Dim(), acts[l]->pCUData(),
                                          (int)acts[l]->Stride(), eo->pCUData(), eo->Dim(), cp.pCUData(),
                                          (int)cp.Stride(), S);
          }
          if (st == TNET_ERR_UNSUPPORTED)
            st = tnet_affine_bwd_colsum(err->pCUData(), err->Dim(), lin->LinearityRO().pCUData(),
                                        lin->LinearityRO().Dim(), acts[l]->pCUData(), (int)acts[l]->Stride(),
                                        eo->pCUData(), eo->Dim(), cp.pCUData(), (int)cp.Stride(), S);
          if (st != TNET_ERR_UNSUPPORTED) {
            TNET_SAFE_CALL(st);
            eo_colsum = true;
          }
        }
      }
      if (!eo_colsum) {
        flush_grad();
        flush();
        KTScope kt("gemm_bwd:" + shape, 2.0 * rows * lin->GetNInputs() * lin->GetNOutputs());
        TNET_SAFE_CALL(tnet_affine_bwd(err->pCUData(), err->Dim(), lin->LinearityRO().pCUData(),
                                       lin->LinearityRO().Dim(), acts[l]->pCUData(), (int)acts[l]->Stride(),
                                       eo->pCUData(), eo->Dim(), 1, S));
      }
    }
    if (top_slabs_ride) {  // no colsum backward launch took the top slab sums
      top_slabs_ride = false;
      err_colsum = top_slabs_launch();
    }
    // the last layer trained here: the held-back update of the layer above and this layer's own are
    // independent (each reads its X, E and writes its own W, b) and no backward GEMM is left -- small ones
    // (both grids in one round over the CUs) go out as ONE launch
    // (with the next bunch's gather on the CUs their tiles leave free, when the trainer handed one over)
    if ((stopper || l == 0) && pend.lin && !exchange && err_colsum && lin->LearnRate() > 0.0f) {
      if (mHasTailGather && !mTailDone &&
          pend.lin->UpdateFromColsumGather(*pend.X, *pend.E, *mColPart[pend.l], lin, acts[l], err, mColPart[l].get(),
                                           mTailGather)) {
        mTailDone = true;
        pend.lin = nullptr;
        break;
      }
      if (pend.lin->UpdatePairFromColsum(*pend.X, *pend.E, *mColPart[pend.l], *lin, *acts[l], *err, *mColPart[l])) {
        pend.lin = nullptr;
        break;
      }
    }
    flush();  // a held-back update no backward GEMM took
    const bool last = stopper || l == 0;
    // a held-back gradient no backward GEMM took (the last layer may still take it, with the gather, below)
    if (!(exchange && last && err_colsum && lin->LearnRate() > 0.0f && mHasTailGather && !mTailDone)) flush_grad();
    if (lin->LearnRate() > 0.0f) {
      if (exchange) {
        lin->SetInput(*acts[l]);
        lin->SetErrorInput(*err);
        if (err_colsum && !last && g_dp_pair) {
          pgrad = lin;  // held back for the next layer's backward GEMM (flushed there or at the next layer)
          pgrad_l = l;
        } else {
          // the step's last gradient GEMM carries the next bunch's gather (when the trainer handed one over) --
          // with the held-back gradient of the layer above in the same launch where both grids fit one round
          CuBiasedLinearity* with = nullptr;  // that held-back layer
          if (err_colsum && last && mHasTailGather && !mTailDone && pgrad &&
              lin->ComputeGradientColsumGather(*mColPart[l], mTailGather, pgrad, mColPart[pgrad_l].get())) {
            mTailDone = true;
            with = pgrad;
            pgrad = nullptr;
          } else {
            flush_grad();
            if (err_colsum && last && mHasTailGather && !mTailDone &&
                lin->ComputeGradientColsumGather(*mColPart[l], mTailGather))
              mTailDone = true;
            else if (err_colsum)
              lin->ComputeGradientColsum(*mColPart[l]);
            else
              lin->ComputeGradient();
          }
          // every trained layer's gradient now exists and none is submitted yet (MLP3: both gradients came from
          // that one launch): no backward GEMM is left to overlap, so the whole reduction goes on the compute
          // stream as one group and the applies right behind it -- no stream hop in or out (a hop is a barrier
          // packet, ~5 us each; the one-rank MLP3 DP step had five)
          CuUpdatableComponent* grp[2];
          int ng = 0;
          if (with) grp[ng++] = with;
          grp[ng++] = lin;
          if (last && n_submitted == 0 && exchange->SubmitInline(grp, ng)) {
            CuBiasedLinearity* lg[2] = {with ? with : lin, lin};
            CuBiasedLinearity::ApplyGradients(lg, ng, grows, exchange);
            n_submitted += ng;
          } else {
            if (with) submit_layer(with, false);
            submit_layer(lin, last);
          }
        }
      } else if (err_colsum) {
        pend.lin = lin;  // held back for the next layer's backward GEMM (flushed there or below)
        pend.X = acts[l];
        pend.E = err;
        pend.l = l;
      } else {
        lin->UpdateFrom(*acts[l], *err);
      }
    }
    if (stopper || l == 0) break;
    err = eo;
    err_colsum = eo_colsum;
  }
  // the step's last update (the stopper's): the next bunch's gather rides on its launch
  if (pend.lin && mHasTailGather && !mTailDone &&
      pend.lin->UpdateFromColsumGather(*pend.X, *pend.E, *mColPart[pend.l], nullptr, nullptr, nullptr, nullptr,
                                       mTailGather)) {
    mTailDone = true;
    pend.lin = nullptr;
  }
  flush();
  flush_grad();
  if (exchange) {
    // the next bunch's gather right behind the last gradient GEMM on the compute stream, so it runs while the
    // last reductions (and their applies) are still in flight instead of after WaitAll at the next step's start
    if (mHasTailGather && !mTailDone) {
      KTScope kt("gather", 2.0 * mTailGather.dy.rows * mTailGather.dy.cols * 4.0);
      TNET_SAFE_CALL(tnet_gather_bunch(mTailGather.y, mTailGather.x, mTailGather.labels_out, mTailGather.labels_in,
                                       mTailGather.copy_from, mTailGather.dy, mTailGather.dx, S));
      mTailDone = true;
    }
    // transports without an apply stream: apply each layer on the compute stream as soon as its own
    // reduction is done (top layer first), overlapping the reductions of the layers below
    const int first = n_submitted - (int)submitted.size();
    for (size_t i = 0; i < submitted.size(); i++) {
      exchange->WaitFor(first + (int)i);
      submitted[i]->ApplyGradient(grows, nullptr, exchange);
      exchange->GatherParams(*submitted[i], first + (int)i, nullptr);
    }
    exchange->WaitAll();
  }
  // restore the component wiring the generic path relies on
  for (int l = 0; l < nl; l++) {
    auto* lin = mNetComponents[2 * l];
    if (l > 0) lin->SetInput(mNetComponents[2 * l - 1]->GetOutput());
    lin->SetErrorInput(mNetComponents[2 * l + 1]->GetErrorOutput());
  }
}

}  // namespace TNet
