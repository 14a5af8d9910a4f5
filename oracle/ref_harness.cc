// ref_harness.cc -- golden-vector generator for the parity tests (TEST INFRASTRUCTURE ONLY).
//
// Links the reference CPU TNetLib/KaldiLib objects (built by oracle/Makefile.ref from the
// read-only sources under /root/reference/src) and drives them exactly the way the
// reference's single-thread training platform does, dumping full-precision results:
//
//   trajectory: the same step loop writing the parameters before / after every step in binary (the
//             reference trajectory of the per-step resync test)
//   step    : per-bunch SGD with TNet --THREADS=1 semantics, i.e. the Platform::Thread
//             bunch loop (src/TNetLib/Platform.h:300-336): clone->Propagate,
//             CrossEntropy::Evaluate, clone->Backpropagate (Gradient()), master
//             AccuGradient/AccuBunchsize/Update(0,1)/ResetBunchsize.
//   train   : the multi-threaded Platform training loop timed around RunTrain (CPU baseline).
//   features: FeatureRepository::ReadFullMatrix + LabelRepository::GenDesiredMatrix over a script,
//             configured as TNetCu does (TNetCu.cc:192-196, 290-314; UserInterface.cc:352-460):
//             every utterance's matrix and class ids, or the exception text of a failing record.
//   shuffle : the cache permutation produced by Cache::Init(seed)+AddData+Randomize
//             (src/TNetLib/Cache.cc:23-192) -- lrand48 + libstdc++ random_shuffle.
//   mlfmatch: KaldiLib's ProcessMask (StkMatch.cc:453-490) and LabelContainer Insert / Find
//             (MlfStream.cc:43-265) answering line commands (the MLF lookup fuzz fixture, make_mlfmatch.py)
//
// It is our own code; no reference source is copied.  Output is raw little-endian float32
// / int32 files plus .nnet text written with 9 significant digits (exact float round trip).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "BiasedLinearity.h"
#include "Nnet.h"
#include "ObjFun.h"
#include "Cache.h"
#include "Matrix.h"
#include "Platform.h"
#include "Features.h"
#include "Labels.h"
#include "Timer.h"
#include "UserInterface.h"
#include "StkMatch.h"
#include "MlfStream.h"

using namespace TNet;

static std::vector<char> slurp(const std::string& path) {
  std::ifstream f(path.c_str(), std::ios::binary);
  if (!f.good()) { std::cerr << "cannot open " << path << "\n"; exit(2); }
  return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static void dump_matrix(const std::string& path, const Matrix<BaseFloat>& m) {
  std::ofstream f(path.c_str(), std::ios::binary);
  for (size_t r = 0; r < m.Rows(); r++)
    for (size_t c = 0; c < m.Cols(); c++) {
      float v = m(r, c);
      f.write((const char*)&v, 4);
    }
}

// step <nnet> <X.f32> <lab.i32> <nIn> <nClasses> <bunch> <nsteps> <lr> <wc> <outdir>
static int cmd_step(int argc, char** argv) {
  if (argc < 12) { std::cerr << "usage: step nnet X lab nIn nCls bunch nsteps lr wc outdir\n"; return 2; }
  std::string nnet_path = argv[2], xpath = argv[3], lpath = argv[4];
  int n_in = atoi(argv[5]), n_cls = atoi(argv[6]), bunch = atoi(argv[7]), nsteps = atoi(argv[8]);
  float lr = (float)atof(argv[9]), wc = (float)atof(argv[10]);
  std::string out = argv[11];

  std::vector<char> xb = slurp(xpath), lb = slurp(lpath);
  const float* X = (const float*)&xb[0];
  const int* L = (const int*)&lb[0];
  size_t nfr = xb.size() / 4 / n_in;
  if ((size_t)bunch * nsteps > nfr) { std::cerr << "not enough frames\n"; return 2; }

  Network nnet;
  nnet.ReadNetwork(nnet_path.c_str());
  nnet.SetLearnRate(lr);
  nnet.SetWeightcost(wc);
  Network* clone = nnet.Clone();
  ObjectiveFunction* obj = ObjectiveFunction::Factory(ObjectiveFunction::CROSS_ENTROPY);

  Matrix<BaseFloat> fea(bunch, n_in), lab(bunch, n_cls), outm, err;
  for (int s = 0; s < nsteps; s++) {
    lab.Zero();
    for (int r = 0; r < bunch; r++) {
      size_t fr = (size_t)s * bunch + r;
      for (int c = 0; c < n_in; c++) fea(r, c) = X[fr * n_in + c];
      if (L[fr] >= 0) lab(r, L[fr]) = 1.0f;   // -1 = unlabeled frame (all-zero target row)
    }
    clone->Propagate(fea, outm);
    obj->Evaluate(outm, lab, &err);
    clone->Backpropagate(err);
    nnet.AccuGradient(*clone, 0, 1);
    nnet.AccuBunchsize(*clone);
    nnet.Update(0, 1);
    nnet.ResetBunchsize();

    std::ostringstream ys, es, ns;
    ys << out << "/Y_" << s << ".f32";
    es << out << "/E_" << s << ".f32";
    ns << out << "/nnet_" << s << ".txt";
    dump_matrix(ys.str(), outm);
    dump_matrix(es.str(), err);
    std::ofstream nf(ns.str().c_str());
    nf.precision(9);
    nnet.WriteNetwork(nf);
  }
  std::ofstream rep((out + "/report.txt").c_str());
  rep.precision(17);
  rep << obj->GetError() << " " << obj->GetFrames() << "\n" << obj->Report();
  delete obj;
  delete clone;
  return 0;
}

// the <biasedlinearity> parameters of a network as float32, in .nnet order per layer: W^T [out x in] row by row,
// then b [out].  The weights are read through pointers to the protected members taken in a derived class
// (well-defined access; nothing of TNetLib is modified)
struct LinearityAccess : public BiasedLinearity {
  static const Matrix<BaseFloat>& W(const BiasedLinearity& c) { return c.*(&LinearityAccess::mLinearity); }
  static const Vector<BaseFloat>& b(const BiasedLinearity& c) { return c.*(&LinearityAccess::mBias); }
};
static void dump_params(std::ofstream& f, Network& nnet) {
  for (int i = 0; i < nnet.Layers(); i++) {
    Component& c = nnet.Layer(i);
    if (c.GetType() != Component::BIASED_LINEARITY) continue;
    const BiasedLinearity& bl = static_cast<const BiasedLinearity&>(c);
    const Matrix<BaseFloat>& W = LinearityAccess::W(bl);  // [in x out]
    const Vector<BaseFloat>& b = LinearityAccess::b(bl);
    std::vector<float> buf(W.Rows() * W.Cols());
    for (size_t o = 0; o < W.Cols(); o++)
      for (size_t r = 0; r < W.Rows(); r++) buf[o * W.Rows() + r] = W(r, o);
    f.write((const char*)&buf[0], buf.size() * 4);
    for (size_t o = 0; o < b.Dim(); o++) {
      float v = b[o];
      f.write((const char*)&v, 4);
    }
  }
}

// trajectory <nnet> <X.f32> <lab.i32> <nIn> <nClasses> <bunch> <nsteps> <lr> <wc> <params.f32> <Y.f32>
// The step loop of `step` (TNet --THREADS=1 semantics), writing the parameters BEFORE every step and after the
// last (nsteps + 1 records of dump_params) and every step's network output: the reference trajectory the
// per-step resync test restarts the GPU network from (tests/test_ex01.py)
static int cmd_trajectory(int argc, char** argv) {
  if (argc < 13) { std::cerr << "usage: trajectory nnet X lab nIn nCls bunch nsteps lr wc params Y\n"; return 2; }
  int n_in = atoi(argv[5]), n_cls = atoi(argv[6]), bunch = atoi(argv[7]), nsteps = atoi(argv[8]);
  float lr = (float)atof(argv[9]), wc = (float)atof(argv[10]);
  std::vector<char> xb = slurp(argv[3]), lb = slurp(argv[4]);
  const float* X = (const float*)&xb[0];
  const int* L = (const int*)&lb[0];
  if ((size_t)bunch * nsteps > xb.size() / 4 / n_in) { std::cerr << "not enough frames\n"; return 2; }
  Network nnet;
  nnet.ReadNetwork(argv[2]);
  nnet.SetLearnRate(lr);
  nnet.SetWeightcost(wc);
  Network* clone = nnet.Clone();
  ObjectiveFunction* obj = ObjectiveFunction::Factory(ObjectiveFunction::CROSS_ENTROPY);
  std::ofstream pf(argv[11], std::ios::binary), yf(argv[12], std::ios::binary);
  Matrix<BaseFloat> fea(bunch, n_in), lab(bunch, n_cls), outm, err;
  dump_params(pf, nnet);
  for (int s = 0; s < nsteps; s++) {
    lab.Zero();
    for (int r = 0; r < bunch; r++) {
      size_t fr = (size_t)s * bunch + r;
      for (int c = 0; c < n_in; c++) fea(r, c) = X[fr * n_in + c];
      if (L[fr] >= 0) lab(r, L[fr]) = 1.0f;
    }
    clone->Propagate(fea, outm);
    obj->Evaluate(outm, lab, &err);
    clone->Backpropagate(err);
    nnet.AccuGradient(*clone, 0, 1);
    nnet.AccuBunchsize(*clone);
    nnet.Update(0, 1);
    nnet.ResetBunchsize();
    for (size_t r = 0; r < outm.Rows(); r++)
      for (size_t c = 0; c < outm.Cols(); c++) {
        float v = outm(r, c);
        yf.write((const char*)&v, 4);
      }
    dump_params(pf, nnet);
  }
  std::cout.precision(17);
  std::cout << obj->GetError() << " " << obj->GetFrames() << "\n";
  delete obj;
  delete clone;
  return 0;
}

// shuffle <seed> <n> <cachesize> <bunch> <out.i32> : emits the row order GetBunch returns
static int cmd_shuffle(int argc, char** argv) {
  if (argc < 7) { std::cerr << "usage: shuffle seed n cachesize bunch out\n"; return 2; }
  long seed = atol(argv[2]);
  int n = atoi(argv[3]), cachesize = atoi(argv[4]), bunch = atoi(argv[5]);
  Cache cache;
  cache.Init(cachesize, bunch, seed);
  Matrix<BaseFloat> fea(n, 1), lab(n, 1);
  for (int i = 0; i < n; i++) { fea(i, 0) = (float)i; lab(i, 0) = 1.0f; }
  cache.AddData(fea, lab);
  cache.Randomize();
  std::ofstream f(argv[6], std::ios::binary);
  Matrix<BaseFloat> f2, l2;
  while (!cache.Empty()) {
    cache.GetBunch(f2, l2);
    for (size_t r = 0; r < f2.Rows(); r++) {
      int v = (int)f2(r, 0);
      f.write((const char*)&v, 4);
    }
  }
  return 0;
}

// train <nnet> <scp> <mlf> <statemap> <lbl_dir> <threads> <bunch> <cache> <lr> <seed>
// The reference's multi-threaded CPU training (Platform::RunTrain, src/TNetLib/Platform.h:143-198:
// one HTK/MLF reader thread + <threads> SGD workers over row slices of each bunch), set up the way
// src/TNet.cc:160-320 sets it up with default feature options, and timed around RunTrain ONLY
// (TNet's own FPS line also counts reading and writing the model text: TNet.cc:321-362).
// Prints "HARNESS_RESULT frames <n> seconds <t>" on stderr.  Used as the CPU baseline of bench.py.
static int cmd_train(int argc, char** argv) {
  if (argc < 12) { std::cerr << "usage: train nnet scp mlf statemap lbl_dir threads bunch cache lr seed\n"; return 2; }
  UserInterface ui;  // no options set: every feature parameter takes its default
  int deriv_order = 0, start_ext = 0, end_ext = 0;
  int* deriv_win = NULL;
  char *cmn_path = NULL, *cmn_file = NULL, *cvn_path = NULL, *cvn_file = NULL;
  const char *cmn_mask = NULL, *cvn_mask = NULL, *cvg_file = NULL;
  int target_kind = ui.GetFeatureParams(&deriv_order, &deriv_win, &start_ext, &end_ext, &cmn_path, &cmn_file,
                                        &cmn_mask, &cvn_path, &cvn_file, &cvn_mask, &cvg_file, "TNET:", 0);
  Platform pl;
  pl.feature_.Init(!TNet::IsBigEndian(), start_ext, end_ext, target_kind, deriv_order, deriv_win, cmn_path,
                   cmn_mask, cvn_path, cvn_mask, cvg_file);
  pl.feature_.AddFileList(argv[3]);
  pl.label_.Init(argv[4], argv[5], argv[6], "lab");
  pl.nnet_.ReadNetwork(argv[2]);
  pl.nnet_.SetLearnRate((float)atof(argv[10]));
  pl.nnet_.SetWeightcost(0.0f);
  pl.obj_fun_ = ObjectiveFunction::Factory(ObjectiveFunction::CROSS_ENTROPY);
  CrossEntropy* xent = dynamic_cast<CrossEntropy*>(pl.obj_fun_);
  xent->SetConfusionMode(CrossEntropy::NO_CONF);
  xent->SetOutputLabelMap(argv[5]);
  pl.bunchsize_ = atoi(argv[8]);
  pl.cachesize_ = atoi(argv[9]);
  pl.randomize_ = true;
  pl.start_frm_ext_ = start_ext;
  pl.end_frm_ext_ = end_ext;
  pl.trace_ = 0;
  pl.crossval_ = false;
  pl.seed_ = atol(argv[11]);
  const int threads = atoi(argv[7]);
  Timer timer;
  timer.Start();
  pl.RunTrain(threads);
  timer.End();
  // on stderr: the worker threads may still be printing to stdout
  std::cerr << "HARNESS_RESULT frames " << pl.obj_fun_->GetFrames() << " seconds " << timer.Val() << std::endl;
  // the measurement is done: leave without running Platform's destructors (the reference's
  // reader/worker teardown intermittently faults at exit, about one run in three here)
  std::cout.flush();
  std::cerr.flush();
  std::_Exit(0);
}

// features <scp> <swap> <start_ext> <end_ext> <TARGETKIND> <mlf|-> <map> <label_dir|-> <label_ext> <outdir>
//          [<CMEANDIR|-> <CMEANMASK|-> <VARSCALEDIR|-> <VARSCALEMASK|-> <VARSCALEFN|->]
// outdir/index.txt: "k rows cols period kind n_labels logical" or "k ERROR <message>" per record;
// outdir/f<k>.f32 (rows x cols), outdir/l<k>.i32 (argmax of each GenDesiredMatrix row)
static int cmd_features(int argc, char** argv) {
  if (argc < 12) { std::cerr << "usage: features scp swap sext eext TARGETKIND mlf map ldir lext outdir\n"; return 2; }
  const bool swap = atoi(argv[3]) != 0;
  const int sext = atoi(argv[4]), eext = atoi(argv[5]);
  int target_kind = FeatureRepository::ReadParmKind(argv[6], false);
  if (target_kind == -1) { std::cerr << "bad TARGETKIND\n"; return 2; }
  // UserInterface::GetFeatureParams without DERIVWINDOWS (UserInterface.cc:444-459)
  int deriv_order = target_kind & PARAMKIND_T ? 3 : target_kind & PARAMKIND_A ? 2 : target_kind & PARAMKIND_D ? 1 : 0;
  int* win = NULL;
  if (deriv_order || target_kind != PARAMKIND_ANON) {
    win = (int*)malloc(3 * sizeof(int));
    win[0] = win[1] = win[2] = 2;
  }
  const std::string mlf = argv[7], map = argv[8], ldir = argv[9], lext = argv[10], out = argv[11];
  // optional: CMEANDIR CMEANMASK VARSCALEDIR VARSCALEMASK VARSCALEFN ("-" = unset), composed into the
  // repository's paths as UserInterface::GetFeatureParams does (UserInterface.cc:385-410: dir + "/")
  std::string cmn_path, cvn_path;
  const char *cmn_mask = NULL, *cvn_mask = NULL, *cvg = NULL;
  if (argc >= 17) {
    if (strcmp(argv[13], "-")) {
      cmn_mask = argv[13];
      cmn_path = strcmp(argv[12], "-") ? std::string(argv[12]) + "/" : std::string();
    }
    if (strcmp(argv[15], "-")) {
      cvn_mask = argv[15];
      cvn_path = strcmp(argv[14], "-") ? std::string(argv[14]) + "/" : std::string();
    }
    if (strcmp(argv[16], "-")) cvg = argv[16];
  }
  FeatureRepository repo;
  repo.Init(swap, sext, eext, target_kind, deriv_order, win, cmn_mask ? cmn_path.c_str() : NULL, cmn_mask,
            cvn_mask ? cvn_path.c_str() : NULL, cvn_mask, cvg);
  repo.AddFileList(argv[2]);
  LabelRepository labels;
  const bool use_mlf = mlf != "-";
  if (use_mlf) labels.Init(mlf.c_str(), map.c_str(), ldir == "-" ? NULL : ldir.c_str(), lext.c_str());
  std::ofstream idx((out + "/index.txt").c_str());
  repo.Rewind();
  for (int k = 0; !repo.EndOfList(); k++, repo.MoveNext()) {
    try {
      Matrix<BaseFloat> m;
      repo.ReadFullMatrix(m);
      std::ostringstream fn;
      fn << out << "/f" << k << ".f32";
      dump_matrix(fn.str(), m);
      int nl = 0;
      if (use_mlf) {
        Matrix<BaseFloat> d;
        labels.GenDesiredMatrix(d, m.Rows() - sext - eext, repo.CurrentHeader().mSamplePeriod,
                                repo.Current().Logical().c_str());
        std::ostringstream ln;
        ln << out << "/l" << k << ".i32";
        std::ofstream lf(ln.str().c_str(), std::ios::binary);
        for (size_t r = 0; r < d.Rows(); r++) {
          int best = -1;
          for (size_t c = 0; c < d.Cols(); c++)
            if (d(r, c) == 1.0f) best = (int)c;
          lf.write((const char*)&best, 4);
        }
        nl = (int)d.Rows();
      }
      idx << k << " " << m.Rows() << " " << m.Cols() << " " << repo.CurrentHeader().mSamplePeriod << " "
          << repo.CurrentHeader().mSampleKind << " " << nl << " " << repo.Current().Logical() << "\n";
    } catch (std::exception& e) {
      std::string msg = e.what();
      for (size_t i = 0; i < msg.size(); i++)
        if (msg[i] == '\n') msg[i] = ' ';
      idx << k << " ERROR " << msg << "\n";
    }
  }
  idx.flush();
  std::_Exit(0);
}

// mlfmatch: line commands on stdin (fields separated by TAB), one answer line per query on stdout
//   M <mask> <label>      ProcessMask(label, mask, sub): "1\t<sub>" or "0"
//   I <pattern> <record>  LabelContainer::Insert(pattern, record) into the current container
//   F <label>             LabelContainer::Find(label): the record's number or -1
//   R                     start a new, empty container
static int cmd_mlfmatch() {
  LabelContainer* box = new LabelContainer();
  std::string line;
  while (std::getline(std::cin, line)) {
    std::vector<std::string> f;
    size_t a = 0;
    for (;;) {
      size_t b = line.find('\t', a);
      f.push_back(line.substr(a, b == std::string::npos ? std::string::npos : b - a));
      if (b == std::string::npos) break;
      a = b + 1;
    }
    if (f[0] == "M" && f.size() == 3) {
      std::string sub;
      const bool ok = ProcessMask(f[2], f[1], sub);
      if (ok) std::cout << "1\t" << sub << "\n";
      else std::cout << "0\n";
    } else if (f[0] == "I" && f.size() == 3) {
      box->Insert(f[1], std::streampos(atol(f[2].c_str())));
    } else if (f[0] == "F" && f.size() == 2) {
      LabelRecord rec;
      if (box->Find(f[1], rec)) std::cout << (long)(std::streamoff)rec.mStreamPos << "\n";
      else std::cout << "-1\n";
    } else if (f[0] == "R") {
      box = new LabelContainer();  // the previous one is left allocated: its destructor is not the subject
    } else {
      std::cerr << "bad command: " << line << "\n";
      return 2;
    }
  }
  std::cout.flush();
  std::_Exit(0);
}

int main(int argc, char** argv) try {
  if (argc < 2) { std::cerr << "modes: step | trajectory | shuffle | train | features | mlfmatch\n"; return 2; }
  if (std::string(argv[1]) == "mlfmatch") return cmd_mlfmatch();
  std::string mode = argv[1];
  if (mode == "step") return cmd_step(argc, argv);
  if (mode == "trajectory") return cmd_trajectory(argc, argv);
  if (mode == "shuffle") return cmd_shuffle(argc, argv);
  if (mode == "train") return cmd_train(argc, argv);
  if (mode == "features") return cmd_features(argc, argv);
  std::cerr << "unknown mode\n";
  return 2;
} catch (std::exception& e) {
  std::cerr << "exception: " << e.what() << "\n";
  return 1;
}
