// capi.cpp -- extern "C" entry points of include/tnet_train.h over the C++ classes.
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>

#include "tnet_train.h"
#include "curbm.h"
#include "curecurrent.h"
#include "htkio.h"
#include "trainer.h"

using namespace TNet;

static thread_local std::string g_last_error;

#define TRY_BEGIN try {
#define TRY_END                              \
  }                                          \
  catch (std::exception & e) {               \
    g_last_error = e.what();                 \
    return TNET_ERR_RUNTIME;                 \
  }                                          \
  return TNET_OK;
#define TRY_END_PTR                          \
  catch (std::exception & e) {               \
    g_last_error = e.what();                 \
    return nullptr;                          \
  }

struct TnetNetwork {
  CuNetwork net;
  CuMatrix<BaseFloat> in_view, out, err_view, tmp_view;
  CuVector<int> lab_view;
  GradExchange* comm = nullptr;
};
struct TnetObjective {
  std::unique_ptr<CuObjectiveFunction> obj;
  CuMatrix<BaseFloat> out_view, des_view, err;
  CuVector<int> lab_view;
};
struct TnetTrainer {
  std::unique_ptr<CuTrainer> t;
};
struct TnetRbmTrainer {
  std::unique_ptr<CuRbmTrainer> t;
};
struct TnetRnnTrainer {
  std::unique_ptr<CuRecurrentTrainer> t;
};
struct TnetFeatureReader {
  std::unique_ptr<tnetio::FeatureReader> r;
  int start_ext = 0, end_ext = 0;
};
struct TnetComm {
  std::unique_ptr<GradExchange> ex;
  RcclExchange* rccl = nullptr;  // one of these two is set
  HostExchange* host = nullptr;
};

extern "C" {

const char* tnet_status_str(int st) {
  switch (st) {
    case TNET_OK: return "ok";
    case TNET_ERR_ARG: return "invalid argument";
    case TNET_ERR_LAUNCH: return "kernel launch failed";
    case TNET_ERR_RUNTIME: return "runtime error";
    case TNET_ERR_UNSUPPORTED: return "unsupported";
    default: return "unknown status";
  }
}

const char* tnet_version(void) { return "tnet_amd 0.1 gfx950 (fp32 MFMA 32x32x2)"; }

const char* tnet_last_error(void) { return g_last_error.c_str(); }

// ---------------------------------------------------------------------------------- runtime
int tnet_device_count(int* n) {
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    g_last_error = hipGetErrorString(e);
    return TNET_ERR_RUNTIME;
  }
  return TNET_OK;
}
int tnet_select_gpu(int id) {
  TRY_BEGIN CuDevice::Instantiate().SelectGPU(id);
  TRY_END
}
int tnet_synchronize(void) {
  TRY_BEGIN CuDevice::Instantiate().Synchronize();
  TRY_END
}
void* tnet_stream(void) {
  try {
    return (void*)CuDevice::Instantiate().Stream();
  } catch (std::exception& e) {
    g_last_error = e.what();
    return nullptr;
  }
}
int tnet_malloc(void** p, size_t bytes) {
  TRY_BEGIN CuDevice::Instantiate();
  TNET_HIP_CALL(hipMalloc(p, bytes));
  TRY_END
}
int tnet_free(void* p) {
  TRY_BEGIN TNET_HIP_CALL(hipFree(p));
  TRY_END
}
int tnet_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  TRY_BEGIN hipStream_t s = CuDevice::Instantiate().Stream();
  TNET_HIP_CALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
  TNET_HIP_CALL(hipStreamSynchronize(s));
  TRY_END
}
int tnet_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  TRY_BEGIN hipStream_t s = CuDevice::Instantiate().Stream();
  TNET_HIP_CALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
  TNET_HIP_CALL(hipStreamSynchronize(s));
  TRY_END
}
int tnet_memcpy_d2d(void* dst, const void* src, size_t bytes) {
  TRY_BEGIN TNET_HIP_CALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, CuDevice::Instantiate().Stream()));
  TRY_END
}
int tnet_memset(void* dst, int value, size_t bytes) {
  TRY_BEGIN TNET_HIP_CALL(hipMemsetAsync(dst, value, bytes, CuDevice::Instantiate().Stream()));
  TRY_END
}
int tnet_set_profile(int on) {
  TRY_BEGIN CuDevice::Instantiate().Profile(on != 0);
  TRY_END
}
int tnet_profile_report(char* buf, int cap) {
  TRY_BEGIN std::ostringstream os;
  CuDevice::Instantiate().PrintProfile(os);
  std::string s = os.str();
  if (cap > 0) {
    std::strncpy(buf, s.c_str(), (size_t)cap - 1);
    buf[cap - 1] = 0;
  }
  TRY_END
}

int tnet_kernel_timing(int on) {
  TRY_BEGIN CuDevice::Instantiate().KernelTiming(on == 2 ? 2 : on != 0 ? 1 : 0);
  TRY_END
}
int tnet_kernel_timing_filter(const char* filter) {
  TRY_BEGIN CuDevice::Instantiate().KernelTimingFilter(filter ? filter : "");
  TRY_END
}
int tnet_kernel_timing_report(char* buf, int cap) {
  TRY_BEGIN std::string s = CuDevice::Instantiate().KTCollect();
  if ((int)s.size() >= cap) Error("tnet_kernel_timing_report: buffer too small");
  std::strncpy(buf, s.c_str(), (size_t)cap);
  TRY_END
}

static hipEvent_t g_t0 = nullptr, g_t1 = nullptr;
int tnet_timer_start(void) {
  TRY_BEGIN if (!g_t0) {
    TNET_HIP_CALL(hipEventCreate(&g_t0));
    TNET_HIP_CALL(hipEventCreate(&g_t1));
  }
  TNET_HIP_CALL(hipEventRecord(g_t0, CuDevice::Instantiate().Stream()));
  TRY_END
}
int tnet_timer_stop(float* ms) {
  TRY_BEGIN TNET_HIP_CALL(hipEventRecord(g_t1, CuDevice::Instantiate().Stream()));
  TNET_HIP_CALL(hipEventSynchronize(g_t1));
  TNET_HIP_CALL(hipEventElapsedTime(ms, g_t0, g_t1));
  TRY_END
}

// ---------------------------------------------------------------------------------- network
TnetNetwork* tnet_net_read(const char* path) {
  try {
    std::unique_ptr<TnetNetwork> h(new TnetNetwork);
    h->net.ReadNetwork(path);
    return h.release();
  }
  TRY_END_PTR
}
TnetNetwork* tnet_net_read_text(const char* text) {
  try {
    std::unique_ptr<TnetNetwork> h(new TnetNetwork);
    std::istringstream is(text);
    h->net.ReadNetwork(is);
    return h.release();
  }
  TRY_END_PTR
}
int tnet_net_write(TnetNetwork* h, const char* path) {
  TRY_BEGIN h->net.WriteNetwork(path);
  TRY_END
}
int tnet_net_free(TnetNetwork* h) {
  TRY_BEGIN delete h;
  TRY_END
}
int tnet_net_num_components(TnetNetwork* h) { return h ? h->net.Layers() : TNET_ERR_ARG; }
int tnet_net_component(TnetNetwork* h, int i, char* tag, int cap, int* n_in, int* n_out) {
  TRY_BEGIN if (i < 0 || i >= h->net.Layers()) Error("component index out of range");
  CuComponent& c = h->net.Layer(i);
  if (tag && cap > 0) {
    std::strncpy(tag, c.GetName(), (size_t)cap - 1);
    tag[cap - 1] = 0;
  }
  if (n_in) *n_in = (int)c.GetNInputs();
  if (n_out) *n_out = (int)c.GetNOutputs();
  TRY_END
}
static CuBiasedLinearity& linear(TnetNetwork* h, int i) {
  if (i < 0 || i >= h->net.Layers()) Error("component index out of range");
  auto* p = dynamic_cast<CuBiasedLinearity*>(&h->net.Layer(i));
  if (!p) Error("component is not <biasedlinearity>");
  return *p;
}
int tnet_net_get_params(TnetNetwork* h, int i, float* W, float* b) {
  TRY_BEGIN CuBiasedLinearity& L = linear(h, i);
  if (W) L.Linearity().CopyToHost(W, L.Linearity().Cols());
  if (b) L.Bias().CopyToHost(b);
  TRY_END
}
int tnet_net_set_params(TnetNetwork* h, int i, const float* W, const float* b) {
  TRY_BEGIN CuBiasedLinearity& L = linear(h, i);
  if (W) {
    CuMatrix<BaseFloat>& M = L.Linearity();
    TNET_HIP_CALL(hipMemcpy2DAsync(M.pCUData(), M.Stride() * 4, W, M.Cols() * 4, M.Cols() * 4, M.Rows(),
                                   hipMemcpyHostToDevice, CuDevice::Instantiate().Stream()));
  }
  if (b) TNET_HIP_CALL(hipMemcpyAsync(L.Bias().pCUData(), b, L.Bias().Dim() * 4, hipMemcpyHostToDevice,
                                      CuDevice::Instantiate().Stream()));
  CuDevice::Instantiate().Synchronize();
  TRY_END
}
int tnet_net_set_learn_rate(TnetNetwork* h, float lr, const char* factors) {
  TRY_BEGIN h->net.SetLearnRate(lr, factors);
  TRY_END
}
int tnet_net_set_momentum(TnetNetwork* h, float mmt) {
  TRY_BEGIN h->net.SetMomentum(mmt);
  TRY_END
}
int tnet_net_set_weightcost(TnetNetwork* h, float wc) {
  TRY_BEGIN h->net.SetWeightcost(wc);
  TRY_END
}
int tnet_net_set_grad_div_frm(TnetNetwork* h, int div) {
  TRY_BEGIN h->net.SetGradDivFrm(div != 0);
  TRY_END
}
int tnet_net_propagate(TnetNetwork* h, const float* dX, int rows, int ldx, float* dY, int ldy) {
  TRY_BEGIN CuMatrix<BaseFloat>::MakeView(h->in_view, const_cast<float*>(dX), rows, h->net.GetNInputs(), ldx);
  h->net.Propagate(h->in_view, h->out);
  if (dY)
    TNET_HIP_CALL(hipMemcpy2DAsync(dY, (size_t)ldy * 4, h->out.pCUData(), h->out.Stride() * 4, h->out.Cols() * 4,
                                   h->out.Rows(), hipMemcpyDeviceToDevice, CuDevice::Instantiate().Stream()));
  TRY_END
}
int tnet_net_backpropagate(TnetNetwork* h, const float* dE, int rows, int lde) {
  TRY_BEGIN CuMatrix<BaseFloat>::MakeView(h->err_view, const_cast<float*>(dE), rows, h->net.GetNOutputs(), lde);
  h->net.Backpropagate(h->err_view);
  TRY_END
}
int tnet_net_train_bunch(TnetNetwork* h, TnetObjective* o, const float* dX, int rows, int ldx, const int* dLabels,
                         int train) {
  TRY_BEGIN CuMatrix<BaseFloat>::MakeView(h->in_view, const_cast<float*>(dX), rows, h->net.GetNInputs(), ldx);
  CuVector<int>::MakeView(h->lab_view, const_cast<int*>(dLabels), rows);
  h->net.TrainBunch(h->in_view, h->lab_view, *o->obj, train != 0, train ? h->comm : nullptr);
  TRY_END
}
int tnet_net_set_comm(TnetNetwork* h, TnetComm* c) {
  TRY_BEGIN h->comm = c ? c->ex.get() : nullptr;
  TRY_END
}
int tnet_net_train_empty(TnetNetwork* h, TnetComm* c, long global_rows) {
  TRY_BEGIN if (!c) Error("tnet_net_train_empty: no communicator");
  c->ex->SetStepRows((size_t)global_rows);
  h->net.TrainEmpty(*c->ex);
  c->ex->SetStepRows(0);
  TRY_END
}
int tnet_net_keep_output(TnetNetwork* h, int keep) {
  TRY_BEGIN h->net.KeepOutput(keep != 0);
  TRY_END
}
int tnet_net_output(TnetNetwork* h, int i, float* host, int ld) {
  TRY_BEGIN if (i < 0 || i >= h->net.Layers()) Error("component index out of range");
  h->net.Layer(i).GetOutput().CopyToHost(host, (size_t)ld);
  TRY_END
}

// -------------------------------------------------------------------------------- objective
TnetObjective* tnet_obj_create(int type) {
  try {
    std::unique_ptr<TnetObjective> h(new TnetObjective);
    h->obj.reset(CuObjectiveFunction::Factory(type == 1 ? CuObjectiveFunction::MEAN_SQUARE_ERROR
                                                        : CuObjectiveFunction::CROSS_ENTROPY));
    return h.release();
  }
  TRY_END_PTR
}
int tnet_obj_free(TnetObjective* o) {
  TRY_BEGIN delete o;
  TRY_END
}
int tnet_obj_evaluate(TnetObjective* o, const float* dOut, int rows, int cols, int ldo, const float* dDes, int ldd,
                      float* dErr, int lde) {
  TRY_BEGIN CuMatrix<BaseFloat>::MakeView(o->out_view, const_cast<float*>(dOut), rows, cols, ldo);
  CuMatrix<BaseFloat>::MakeView(o->des_view, const_cast<float*>(dDes), rows, cols, ldd);
  CuMatrix<BaseFloat> err;
  CuMatrix<BaseFloat>::MakeView(err, dErr, rows, cols, lde);
  o->obj->Evaluate(o->out_view, o->des_view, err);
  TRY_END
}
int tnet_obj_evaluate_labels(TnetObjective* o, const float* dOut, int rows, int cols, int ldo, const int* dLabels,
                             float* dErr, int lde) {
  TRY_BEGIN CuMatrix<BaseFloat>::MakeView(o->out_view, const_cast<float*>(dOut), rows, cols, ldo);
  CuVector<int>::MakeView(o->lab_view, const_cast<int*>(dLabels), rows);
  CuMatrix<BaseFloat> err;
  CuMatrix<BaseFloat>::MakeView(err, dErr, rows, cols, lde);
  o->obj->EvaluateLabels(o->out_view, o->lab_view, err);
  TRY_END
}
int tnet_obj_stats(TnetObjective* o, double* error, long* frames, double* correct) {
  TRY_BEGIN if (error) *error = o->obj->GetError();
  if (correct) *correct = o->obj->GetCorrect();
  if (frames) *frames = (long)o->obj->GetFrames();
  TRY_END
}
int tnet_obj_report(TnetObjective* o, char* buf, int cap) {
  TRY_BEGIN std::string s = o->obj->Report();
  if (cap > 0) {
    std::strncpy(buf, s.c_str(), (size_t)cap - 1);
    buf[cap - 1] = 0;
  }
  TRY_END
}
int tnet_obj_reset(TnetObjective* o) {
  TRY_BEGIN o->obj->Reset();
  TRY_END
}

// ---------------------------------------------------------------------------------- trainer
TnetTrainer* tnet_trainer_create(TnetNetwork* net, TnetObjective* obj, int bunchsize, int cachesize, long seed,
                                 int randomize, int crossval) {
  try {
    TrainerOptions opt;
    opt.bunchsize = (size_t)bunchsize;
    opt.cachesize = (size_t)cachesize;
    opt.seed = seed;
    opt.randomize = randomize != 0;
    opt.crossval = crossval != 0;
    std::unique_ptr<TnetTrainer> h(new TnetTrainer);
    h->t.reset(new CuTrainer(&net->net, obj->obj.get(), opt));
    return h.release();
  }
  TRY_END_PTR
}
int tnet_trainer_free(TnetTrainer* t) {
  TRY_BEGIN delete t;
  TRY_END
}
int tnet_trainer_add_utterance(TnetTrainer* t, const float* feats, int rows, int cols, int ld, const int* labels) {
  TRY_BEGIN t->t->AddUtterance(feats, (size_t)rows, (size_t)cols, (size_t)ld, labels);
  TRY_END
}
int tnet_trainer_finish(TnetTrainer* t) {
  TRY_BEGIN t->t->Finish();
  TRY_END
}
long tnet_trainer_steps(TnetTrainer* t) { return t ? t->t->Steps() : -1; }
int tnet_debug_fail_train_bunch(long n) {
  TRY_BEGIN CuNetwork::DebugFailTrainBunch(n < 0 ? 0 : n);
  TRY_END
}
int tnet_trainer_replay(TnetTrainer* t, long n) {
  TRY_BEGIN t->t->Replay(n);
  TRY_END
}
long tnet_trainer_prefill(TnetTrainer* t, const float* feats, int rows, int cols, int ld, const int* labels) {
  try {
    return (long)t->t->Prefill(feats, (size_t)rows, (size_t)cols, (size_t)ld, labels);
  } catch (std::exception& e) {
    g_last_error = e.what();
    return TNET_ERR_RUNTIME;
  }
}
int tnet_trainer_set_comm(TnetTrainer* t, TnetComm* c) {
  TRY_BEGIN t->t->SetExchange(c ? c->ex.get() : nullptr);
  TRY_END
}
int tnet_trainer_set_transform(TnetTrainer* t, TnetNetwork* transform, int start_ext, int end_ext) {
  TRY_BEGIN if (start_ext < 0 || end_ext < 0) Error("tnet_trainer_set_transform: negative frame extension");
  t->t->SetTransform(transform ? &transform->net : nullptr, (size_t)start_ext, (size_t)end_ext);
  TRY_END
}
long tnet_trainer_empty_steps(TnetTrainer* t) { return t ? t->t->EmptySteps() : -1; }
int tnet_trainer_trace(TnetTrainer* t, int trace) {
  TRY_BEGIN t->t->Cache().Trace(trace);
  TRY_END
}

// ------------------------------------------------------------------------- host front end
TnetFeatureReader* tnet_reader_create(const char* scp, int swap, int start_ext, int end_ext, int target_kind,
                                      int deriv_order, const int* deriv_win, const char* mlf, const char* label_map,
                                      const char* label_dir, const char* label_ext, int threads, int depth) {
  return tnet_reader_create_norm(scp, swap, start_ext, end_ext, target_kind, deriv_order, deriv_win, mlf, label_map,
                                 label_dir, label_ext, nullptr, nullptr, nullptr, nullptr, nullptr, threads, depth);
}
TnetFeatureReader* tnet_reader_create_norm(const char* scp, int swap, int start_ext, int end_ext, int target_kind,
                                           int deriv_order, const int* deriv_win, const char* mlf,
                                           const char* label_map, const char* label_dir, const char* label_ext,
                                           const char* cmn_dir, const char* cmn_mask, const char* cvn_dir,
                                           const char* cvn_mask, const char* cvg_file, int threads, int depth) {
  try {
    if (!scp) Error("tnet_reader_create: no script file");
    if (start_ext < 0 || end_ext < 0) Error("tnet_reader_create: negative frame extension");
    if (mlf && !label_map) Error("Output label map is missing [-m]");
    tnetio::FeatureConfig cfg;
    cfg.swap = swap != 0;
    cfg.startExt = start_ext;
    cfg.endExt = end_ext;
    cfg.targetKind = target_kind;
    cfg.derivOrder = deriv_order;
    if (deriv_win)
      for (int i = 0; i < deriv_order; i++) cfg.derivWin.push_back(deriv_win[i]);
    cfg.cmn = cmn_mask != nullptr;
    cfg.cvn = cvn_mask != nullptr;
    cfg.cvg = cvg_file != nullptr;
    if (cmn_dir) cfg.cmnDir = cmn_dir;
    if (cmn_mask) cfg.cmnMask = cmn_mask;
    if (cvn_dir) cfg.cvnDir = cvn_dir;
    if (cvn_mask) cfg.cvnMask = cvn_mask;
    if (cvg_file) cfg.cvgFile = cvg_file;
    std::shared_ptr<const tnetio::MlfLabels> labels;
    if (mlf) labels = std::make_shared<tnetio::MlfLabels>(mlf, label_map, label_dir, label_ext);
    std::unique_ptr<TnetFeatureReader> h(new TnetFeatureReader);
    h->r.reset(new tnetio::FeatureReader(scp, cfg, labels, threads, depth));
    h->start_ext = start_ext;
    h->end_ext = end_ext;
    return h.release();
  }
  TRY_END_PTR
}
int tnet_reader_free(TnetFeatureReader* r) {
  delete r;
  return TNET_OK;
}
long tnet_reader_size(TnetFeatureReader* r) { return r ? (long)r->r->Size() : -1; }
int tnet_reader_next(TnetFeatureReader* r, const float** feats, int* rows, int* cols, const int** labels,
                     int* n_labels, int* samp_period, int* kind, char* logical, int logical_cap) {
  try {
    if (!r) Error("tnet_reader_next: null reader");
    const tnetio::Utterance* u = r->r->Next();
    if (!u) return 0;
    if (feats) *feats = u->feats.data();
    if (rows) *rows = u->rows;
    if (cols) *cols = u->cols;
    if (labels) *labels = u->labels.empty() ? nullptr : u->labels.data();
    if (n_labels) *n_labels = (int)u->labels.size();
    if (samp_period) *samp_period = u->samplePeriod;
    if (kind) *kind = u->kind;
    if (logical && logical_cap > 0) {
      std::strncpy(logical, u->logical.c_str(), (size_t)logical_cap - 1);
      logical[logical_cap - 1] = '\0';
    }
    return 1;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return TNET_ERR_RUNTIME;
  }
}
int tnet_reader_rewind(TnetFeatureReader* r) {
  TRY_BEGIN if (!r) Error("tnet_reader_rewind: null reader");
  r->r->Rewind();
  TRY_END
}
int tnet_mask_match(const char* mask, const char* label, char* captured, int cap) {
  TRY_BEGIN if (!mask || !label || (cap > 0 && !captured)) Error("tnet_mask_match: null argument");
  std::string sub;
  const bool ok = tnetio::LabelMask::ForPath(mask).Matches(tnetio::LabelMask::AsPath(label), &sub);
  if (cap > 0) {
    const size_t n = std::min(sub.size(), (size_t)cap - 1);
    std::memcpy(captured, sub.data(), n);
    captured[n] = '\0';
  }
  return ok ? 1 : 0;
  TRY_END
}

int tnet_mlf_lookup(const char* const* patterns, int n_patterns, const char* const* labels, int n_labels,
                    int* rec_out) {
  TRY_BEGIN if (n_patterns < 0 || n_labels < 0 || (n_patterns && !patterns) || (n_labels && (!labels || !rec_out)))
      Error("tnet_mlf_lookup: bad arguments");
  tnetio::LabelIndex index;
  for (int k = 0; k < n_patterns; k++) index.Insert(patterns[k] ? patterns[k] : "", (size_t)k);
  for (int i = 0; i < n_labels; i++) {
    size_t rec = 0;
    rec_out[i] = index.Find(labels[i] ? labels[i] : "", &rec) ? (int)rec : -1;
  }
  TRY_END
}

int tnet_htk_read(const char* record, int swap, int start_ext, int end_ext, float* out, long cap, int* rows, int* cols,
                  int* samp_period, int* kind) {
  TRY_BEGIN if (!record) Error("tnet_htk_read: no record");
  tnetio::FeatureConfig cfg;
  cfg.swap = swap != 0;
  cfg.startExt = start_ext;
  cfg.endExt = end_ext;
  int tk = cfg.targetKind, dord = cfg.derivOrder;
  tnetio::Utterance u;
  tnetio::ReadHtkFeatures(tnetio::ParseFileRecord(record), cfg, tk, dord, u);
  if (rows) *rows = u.rows;
  if (cols) *cols = u.cols;
  if (samp_period) *samp_period = u.samplePeriod;
  if (kind) *kind = u.kind;
  if (out) {
    if (cap < (long)u.feats.size()) Error("tnet_htk_read: output buffer too small");
    std::memcpy(out, u.feats.data(), u.feats.size() * sizeof(float));
  }
  TRY_END
}
long tnet_trainer_add_reader(TnetTrainer* t, TnetFeatureReader* r, long max_utts) {
  try {
    if (!t || !r) Error("tnet_trainer_add_reader: null handle");
    long frames = 0;
    for (long n = 0; max_utts < 0 || n < max_utts; n++) {
      const tnetio::Utterance* u = r->r->Next();
      if (!u) break;
      if (u->labels.empty()) Error("tnet_trainer_add_reader: the reader has no labels (no MLF)");
      const std::string bad = tnetio::CheckDataError(*u);  // feats_host.CheckData (TNetCu.cc:386)
      if (!bad.empty()) Error(bad);
      t->t->AddUtteranceExtended(u->feats.data(), (size_t)u->rows, (size_t)u->cols, (size_t)u->cols, u->labels.data(),
                                 (size_t)r->start_ext, (size_t)r->end_ext);
      frames += (long)u->labels.size();
    }
    return frames;
  } catch (std::exception& e) {
    g_last_error = e.what();
    return TNET_ERR_RUNTIME;
  }
}

// ------------------------------------------------------------------------------------ RBM
static CuRbm& rbm_layer(TnetNetwork* h, int i) {
  if (i < 0 || i >= h->net.Layers()) Error("component index out of range");
  auto* p = dynamic_cast<CuRbm*>(&h->net.Layer(i));
  if (!p) Error("component is not <rbm>");
  return *p;
}
int tnet_net_rbm_get(TnetNetwork* h, int i, float* W, float* vb, float* hb, int* types) {
  TRY_BEGIN CuRbm& R = rbm_layer(h, i);
  if (W) R.VisHid().CopyToHost(W, R.VisHid().Cols());
  if (vb) R.VisBias().CopyToHost(vb);
  if (hb) R.HidBias().CopyToHost(hb);
  if (types) {
    types[0] = R.VisType() == CuRbm::BERNOULLI ? 0 : 1;
    types[1] = R.HidType() == CuRbm::BERNOULLI ? 0 : 1;
  }
  TRY_END
}
int tnet_net_rbm_set(TnetNetwork* h, int i, const float* W, const float* vb, const float* hb, int vis_type,
                     int hid_type) {
  TRY_BEGIN CuRbm& R = rbm_layer(h, i);
  if (W) R.VisHid().CopyFromHost(W, R.VisHid().Rows(), R.VisHid().Cols(), R.VisHid().Cols());
  if (vb) R.VisBias().CopyFromHost(vb, R.VisBias().Dim());
  if (hb) R.HidBias().CopyFromHost(hb, R.HidBias().Dim());
  if (vis_type >= 0 && hid_type >= 0)
    R.SetUnitTypes(vis_type == 0 ? CuRbm::BERNOULLI : CuRbm::GAUSSIAN, hid_type == 0 ? CuRbm::BERNOULLI : CuRbm::GAUSSIAN);
  CuDevice::Instantiate().Synchronize();
  TRY_END
}
int tnet_net_rbm_update(TnetNetwork* h, int i, const float* pos_vis, const float* pos_hid, const float* neg_vis,
                        const float* neg_hid, int rows, int ldv, int ldh) {
  TRY_BEGIN CuRbm& R = rbm_layer(h, i);
  CuMatrix<BaseFloat> pv, ph, nv, nh;
  const size_t V = R.GetNInputs(), H = R.GetNOutputs();
  CuMatrix<BaseFloat>::MakeView(pv, const_cast<float*>(pos_vis), rows, V, ldv);
  CuMatrix<BaseFloat>::MakeView(ph, const_cast<float*>(pos_hid), rows, H, ldh);
  CuMatrix<BaseFloat>::MakeView(nv, const_cast<float*>(neg_vis), rows, V, ldv);
  CuMatrix<BaseFloat>::MakeView(nh, const_cast<float*>(neg_hid), rows, H, ldh);
  R.RbmUpdate(pv, ph, nv, nh);
  TRY_END
}
TnetRbmTrainer* tnet_rbm_trainer_create(TnetNetwork* net, int bunchsize, int cachesize, long seed, int randomize,
                                        float lr, float mmt, float wc) {
  try {
    // TRbmCu.cc:221-243: the network holds exactly one <rbm>; lr / momentum / weight cost set on it
    if (net->net.Layers() != 1) Error("Number of layers must be 1");
    CuRbm& R = rbm_layer(net, 0);
    R.LearnRate(lr);
    R.Momentum(mmt);
    R.Weightcost(wc);
    RbmTrainerOptions opt;
    opt.bunchsize = (size_t)bunchsize;
    opt.cachesize = (size_t)cachesize;
    opt.seed = seed;
    opt.randomize = randomize != 0;
    std::unique_ptr<TnetRbmTrainer> h(new TnetRbmTrainer);
    h->t.reset(new CuRbmTrainer(&R, opt));
    return h.release();
  }
  TRY_END_PTR
}
int tnet_rbm_trainer_free(TnetRbmTrainer* t) {
  TRY_BEGIN delete t;
  TRY_END
}
int tnet_rbm_trainer_add_utterance(TnetRbmTrainer* t, const float* feats, int rows, int cols, int ld) {
  TRY_BEGIN t->t->AddUtterance(feats, (size_t)rows, (size_t)cols, (size_t)ld);
  TRY_END
}
int tnet_rbm_trainer_finish(TnetRbmTrainer* t) {
  TRY_BEGIN t->t->Finish();
  TRY_END
}
long tnet_rbm_trainer_steps(TnetRbmTrainer* t) { return t ? t->t->Steps() : -1; }
int tnet_rbm_trainer_stats(TnetRbmTrainer* t, double* mse, long* frames) {
  TRY_BEGIN if (mse) *mse = t->t->Mse().GetError();
  if (frames) *frames = (long)t->t->Mse().GetFrames();
  TRY_END
}
int tnet_rbm_trainer_report(TnetRbmTrainer* t, char* buf, int cap) {
  TRY_BEGIN std::string s = t->t->Mse().Report();
  if (cap > 0) {
    std::strncpy(buf, s.c_str(), (size_t)cap - 1);
    buf[cap - 1] = 0;
  }
  TRY_END
}
long tnet_rbm_trainer_prefill(TnetRbmTrainer* t, const float* feats, int rows, int cols, int ld) {
  try {
    return (long)t->t->Prefill(feats, (size_t)rows, (size_t)cols, (size_t)ld);
  } catch (std::exception& e) {
    g_last_error = e.what();
    return -1;
  }
}
int tnet_rbm_trainer_replay(TnetRbmTrainer* t, long n) {
  TRY_BEGIN t->t->Replay(n);
  TRY_END
}

// ------------------------------------------------------------------------------ recurrent
static CuRecurrent& rnn_layer(TnetNetwork* h, int i) {
  if (i < 0 || i >= h->net.Layers()) Error("component index out of range");
  auto* p = dynamic_cast<CuRecurrent*>(&h->net.Layer(i));
  if (!p) Error("component is not <recurrent>");
  return *p;
}
int tnet_net_recurrent_get(TnetNetwork* h, int i, float* W, float* b) {
  TRY_BEGIN CuRecurrent& R = rnn_layer(h, i);
  if (W) R.Linearity().CopyToHost(W, R.Linearity().Cols());
  if (b) R.Bias().CopyToHost(b);
  TRY_END
}
int tnet_net_recurrent_set(TnetNetwork* h, int i, const float* W, const float* b) {
  TRY_BEGIN CuRecurrent& R = rnn_layer(h, i);
  if (W) R.Linearity().CopyFromHost(W, R.Linearity().Rows(), R.Linearity().Cols(), R.Linearity().Cols());
  if (b) R.Bias().CopyFromHost(b, R.Bias().Dim());
  CuDevice::Instantiate().Synchronize();
  TRY_END
}
TnetRnnTrainer* tnet_rnn_trainer_create(TnetNetwork* net, TnetObjective* obj, int bptt, int crossval) {
  try {
    std::unique_ptr<TnetRnnTrainer> h(new TnetRnnTrainer);
    h->t.reset(new CuRecurrentTrainer(&net->net, obj->obj.get(), bptt, crossval != 0));
    return h.release();
  }
  TRY_END_PTR
}
int tnet_rnn_trainer_free(TnetRnnTrainer* t) {
  TRY_BEGIN delete t;
  TRY_END
}
int tnet_rnn_trainer_utterance(TnetRnnTrainer* t, const float* feats, int rows, int cols, int ld, const int* labels) {
  TRY_BEGIN t->t->TrainUtterance(feats, (size_t)rows, (size_t)cols, (size_t)ld, labels);
  TRY_END
}
long tnet_rnn_trainer_frames(TnetRnnTrainer* t) { return t ? t->t->Frames() : -1; }

// -------------------------------------------------------------------------------------- DP
int tnet_comm_unique_id(char out[128]) {
  TRY_BEGIN RcclExchange::UniqueId(out);
  TRY_END
}
TnetComm* tnet_comm_create(int rank, int world, const char id[128]) {
  try {
    std::unique_ptr<TnetComm> h(new TnetComm);
    h->rccl = new RcclExchange(rank, world, id);
    h->ex.reset(h->rccl);
    return h.release();
  }
  TRY_END_PTR
}
TnetComm* tnet_comm_create_host(int rank, int world, tnet_host_allreduce_fn fn, void* user) {
  try {
    if (!fn || world < 1 || rank < 0 || rank >= world) Error("tnet_comm_create_host: bad arguments");
    std::unique_ptr<TnetComm> h(new TnetComm);
    h->host = new HostExchange(rank, world, fn, user);
    h->ex.reset(h->host);
    return h.release();
  }
  TRY_END_PTR
}
int tnet_comm_set_step_rows(TnetComm* c, long global_rows) {
  TRY_BEGIN if (global_rows < 0) Error("tnet_comm_set_step_rows: negative row count");
  c->ex->SetStepRows((size_t)global_rows);
  TRY_END
}
int tnet_dp_plan_round(TnetComm* c, long n, int final, long* steps, int* ranks_at_step, long cap, int* all_final) {
  TRY_BEGIN DpRoundPlan plan = DpPlanRound(*c->ex, n, final != 0);
  *steps = plan.steps;
  *all_final = plan.all_final ? 1 : 0;
  if (plan.steps > cap) Error("tnet_dp_plan_round: ranks_at_step capacity too small");
  for (long j = 0; j < plan.steps; j++) ranks_at_step[j] = plan.ranks_at_step[(size_t)j];
  TRY_END
}
int tnet_dp_shard_ranges(long n, int rank, int world, long* lo, long* hi, int* count) {
  TRY_BEGIN if (n < 0 || world < 1 || rank < 0 || rank >= world || !lo || !hi || !count)
      Error("tnet_dp_shard_ranges: bad arguments");
  *count = GradExchange::ShardRanges(n, rank, world, lo, hi);
  TRY_END
}
int tnet_comm_free(TnetComm* c) {
  TRY_BEGIN delete c;
  TRY_END
}
int tnet_comm_allreduce_host(TnetComm* c, double* v, int n) {
  TRY_BEGIN c->ex->AllReduceHost(v, n);
  TRY_END
}
int tnet_comm_capture(TnetComm* c, int on) {
  TRY_BEGIN if (!c) Error("tnet_comm_capture: no communicator");
  c->ex->ArmCapture(on != 0);
  TRY_END
}
long tnet_comm_captured(TnetComm* c) {
  if (!c) return -1;
  try {
    return (long)c->ex->Captured().size();  // the first call reads the armed step's device copies back
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return -1;
  }
}
int tnet_comm_captured_block(TnetComm* c, long i, float* local, float* reduced, long cap, long* n) {
  TRY_BEGIN if (!c || !n || i < 0 || i >= (long)c->ex->Captured().size()) Error("tnet_comm_captured_block: bad arguments");
  const GradExchange::CapturedBlock& b = c->ex->Captured()[(size_t)i];
  *n = (long)b.local.size();
  if (local || reduced) {
    if (cap < *n || !local || !reduced) Error("tnet_comm_captured_block: buffers too small");
    std::memcpy(local, b.local.data(), b.local.size() * sizeof(float));
    std::memcpy(reduced, b.reduced.data(), b.reduced.size() * sizeof(float));
  }
  TRY_END
}
int tnet_comm_transport_ranks(TnetComm* c, int* ranks) {
  TRY_BEGIN if (!c || !ranks) Error("tnet_comm_transport_ranks: bad arguments");
  *ranks = c->ex->TransportRanks();
  TRY_END
}
int tnet_comm_allreduce_device(TnetComm* c, float* dbuf, long n) {
  TRY_BEGIN if (c->rccl) c->rccl->AllReduceDevice(dbuf, (size_t)n);
  else c->host->AllReduceDevice(dbuf, (size_t)n);
  TRY_END
}

}  // extern "C"
