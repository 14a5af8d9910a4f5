// htkio.cpp -- native HTK / MLF intake with read-ahead (see htkio.h for the reference map).
#include "htkio.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

namespace tnetio {

namespace {

[[noreturn]] void Fail(const std::string& msg) { throw std::runtime_error(msg); }

std::string Trim(const std::string& s) {
  size_t b = s.find_first_not_of(" \t\r\n"), e = s.find_last_not_of(" \t\r\n");
  return b == std::string::npos ? std::string() : s.substr(b, e - b + 1);
}

inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
inline uint16_t bswap16(uint16_t v) { return __builtin_bswap16(v); }

// src/KaldiLib/Features.cc:21-37 + 272-292
std::string ParmKindStr(unsigned k) {
  static const char* names[13] = {"WAVEFORM", "LPC", "LPREFC", "LPCEPSTRA", "LPDELCEP", "IREFC", "MFCC",
                                  "FBANK", "MELSPEC", "USER", "DISCRETE", "PLP", "ANON"};
  if ((k & 0x3F) >= 13) return "";
  std::string s = names[k & 0x3F];
  const std::pair<unsigned, const char*> q[] = {{kParmE, "_E"}, {kParmN, "_N"}, {kParmD, "_D"}, {kParmA, "_A"},
                                                {kParmC, "_C"}, {kParmZ, "_Z"}, {010000, "_K"}, {kParm0, "_0"},
                                                {040000, "_V"}, {kParmT, "_T"}};
  for (auto& p : q)
    if (k & p.first) s += p.second;
  return s;
}

struct Fd {
  int fd;
  explicit Fd(int f) : fd(f) {}
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

HtkHeader DecodeHeader(const unsigned char* b, bool swap) {
  HtkHeader h;
  memcpy(&h.nSamples, b, 4);
  memcpy(&h.samplePeriod, b + 4, 4);
  memcpy(&h.sampleSize, b + 8, 2);
  memcpy(&h.sampleKind, b + 10, 2);
  if (swap) {
    h.nSamples = (int32_t)bswap32((uint32_t)h.nSamples);
    h.samplePeriod = (int32_t)bswap32((uint32_t)h.samplePeriod);
    h.sampleSize = (int16_t)bswap16((uint16_t)h.sampleSize);
    h.sampleKind = bswap16(h.sampleKind);
  }
  return h;
}

// "name[s,e]" -> name, s, e (Features.cc:1045-1054: the suffix must end the string)
bool SplitRange(std::string& name, int& from, int& to) {
  size_t p = name.rfind('[');
  if (p == std::string::npos) return false;
  int n = 0;
  if (sscanf(name.c_str() + p, "[%d,%d]%n", &from, &to, &n) != 2 || name[p + n] != '\0') return false;
  name.erase(p);
  return true;
}


// One frame of a parameter kind: order + 1 blocks (statics, then deltas, accelerations, third
// differences), each block `base` coefficients followed by C0 (_0) and the energy (_E) when the kind has
// them; _N leaves the C0 / energy values out of the static block.
struct FrameLayout {
  bool c0 = false, energy = false;
  int suppressed = 0;  // static values left out by _N
  int order = 0;       // derivative blocks

  static FrameLayout OfKind(int kind) {
    FrameLayout l;
    l.c0 = (kind & kParm0) != 0;
    l.energy = (kind & kParmE) != 0;
    l.suppressed = (kind & kParmN) ? l.Extras() : 0;
    l.order = (kind & kParmT) ? 3 : (kind & kParmA) ? 2 : (kind & kParmD) ? 1 : 0;
    return l;
  }
  int Extras() const { return (int)c0 + (int)energy; }
  int Block(int base) const { return base + Extras(); }
  int Width(int base) const { return Block(base) * (order + 1) - suppressed; }
  int BaseFromWidth(int values) const { return (values + suppressed) / (order + 1) - Extras(); }
  // the first `blocks` + 1 blocks of this layout and of t hold the same values in the same places
  bool SameValues(const FrameLayout& t, int blocks) const {
    return blocks == order && blocks == t.order && c0 == t.c0 && energy == t.energy && suppressed == t.suppressed;
  }
  // Column of the target row each value of a frame of this layout is written to, blocks 0..blocks.  A C0 /
  // energy value the target does not keep is written where the next kept value goes (so it is replaced),
  // or past the kept columns at the end of the row (the derivative columns computed afterwards replace it,
  // a column past the row is dropped) -- the reference's decode into a row with a trailing cursor.
  std::vector<int> PlacementIn(const FrameLayout& t, int base, int blocks) const {
    std::vector<int> col;
    int at = 0;
    for (int b = 0; b <= blocks; b++) {
      for (int k = 0; k < base; k++) col.push_back(at++);
      const bool statics = b == 0;
      const bool src_has[2] = {c0 && !(statics && suppressed), energy && !(statics && suppressed)};
      const bool trg_has[2] = {t.c0 && !(statics && t.suppressed), t.energy && !(statics && t.suppressed)};
      for (int x = 0; x < 2; x++) {
        if (src_has[x]) col.push_back(at);
        if (trg_has[x]) at++;
      }
    }
    return col;
  }
};

// Whether frames of layout s (base kind sb) convert to layout t (base kind tb): C0 and energy cannot be
// made up, a value _N left out of the file cannot come back, _N needs a derivative block to keep the value
// in, derivatives of a file with suppressed statics cannot be computed, and the base kinds must agree
// unless the file's is ANON.
bool Convertible(const FrameLayout& s, const FrameLayout& t, int sb, int tb) {
  if ((t.energy && !s.energy) || (t.c0 && !s.c0)) return false;
  if (s.suppressed && !t.suppressed) return false;
  if (t.suppressed && t.order == 0) return false;
  if (s.suppressed && s.order == 0 && t.order > 0) return false;
  return sb == tb || sb == kParmAnon;
}
}  // namespace

FileRecord ParseFileRecord(const std::string& line) {
  FileRecord r;
  r.logical = line;
  std::replace(r.logical.begin(), r.logical.end(), '\\', '/');
  size_t p = r.logical.find('{');
  if (p != std::string::npos) {
    std::istringstream ss(r.logical.substr(p + 1));
    ss >> r.weight;
    r.logical.erase(p);
  }
  p = r.logical.find('=');
  if (p != std::string::npos) {
    r.physical = Trim(r.logical.substr(p + 1));
    r.logical = Trim(r.logical.substr(0, p));
  } else {
    r.logical = Trim(r.logical);
    r.physical = r.logical;
  }
  return r;
}

HtkHeader ReadHtkHeader(const std::string& physical, bool swap, const std::string& base) {
  std::string name = physical;
  int a, b;
  SplitRange(name, a, b);
  const std::string where = (!base.empty() && !name.empty() && name[0] != '/') ? base + "/" + name : name;
  Fd f(open(where.c_str(), O_RDONLY));
  if (f.fd < 0) Fail("Cannot open feature file: '" + name + "'");
  unsigned char hb[12];
  if (pread(f.fd, hb, 12, 0) != 12) Fail("Invalid HTK header in feature file: '" + name + "'");
  return DecodeHeader(hb, swap);
}

// CMEANDIR / VARSCALEDIR / VARSCALEFN normalisation of a read matrix (Features.cc:1352-1410; defined below)
void ApplyCepsNorm(const FeatureConfig& cfg, const std::string& logical, int targetKind, int derivOrder, int coefs,
                   int trg_N, int trg_vec, int tot, float* M);

void ReadHtkFeatures(const FileRecord& rec, const FeatureConfig& cfg, int& targetKind, int& derivOrder,
                     Utterance& out) {
  std::string name = rec.physical;
  int from_frame = 0, to_frame = 0;
  const bool ranged = SplitRange(name, from_frame, to_frame);
  std::string where = name;  // the file opened: relative names against the directory of the record's creation
  if (!rec.base.empty() && !name.empty() && name[0] != '/') where = rec.base + "/" + name;

  Fd f(open(where.c_str(), O_RDONLY));
  if (f.fd < 0) Fail("Cannot open feature file: '" + name + "'");
  unsigned char hb[12];
  if (pread(f.fd, hb, 12, 0) != 12) Fail("Invalid HTK header in feature file: '" + name + "'");
  HtkHeader h = DecodeHeader(hb, cfg.swap);
  if (h.samplePeriod < 0 || h.samplePeriod > 100000 || h.nSamples < 0 || h.sampleSize < 0)
    Fail("Invalid HTK header in feature file: '" + name + "'");

  int comp = h.sampleKind & kParmC;
  std::vector<float> A, B;
  if (comp) {  // scale and bias vectors follow the header (Features.cc:1086-1108)
    const int n = h.sampleSize / 2;
    A.resize(n);
    B.resize(n);
    std::vector<uint32_t> raw(2 * (size_t)n);
    if (pread(f.fd, raw.data(), raw.size() * 4, 12) != (ssize_t)(raw.size() * 4))
      Fail("Cannot read feature file: '" + name + "'");
    for (auto& v : raw)
      if (cfg.swap) v = bswap32(v);
    memcpy(A.data(), raw.data(), n * 4);
    memcpy(B.data(), raw.data() + n, n * 4);
    h.nSamples -= 2 * 4 / 2;
  }
  if (!ranged) {
    from_frame = 0;
    to_frame = h.nSamples - 1;
  }

  h.sampleKind &= ~kParmC;
  const FrameLayout src = FrameLayout::OfKind(h.sampleKind);
  if (targetKind == kParmAnon) targetKind = h.sampleKind;  // ANON: the file's kind, qualifiers included
  else if ((targetKind & 077) == kParmAnon) targetKind = (targetKind & ~077) | (h.sampleKind & 077);
  FrameLayout trg = FrameLayout::OfKind(targetKind);

  const int value_bytes = comp ? 2 : 4;
  const int coefs = src.BaseFromWidth(h.sampleSize / value_bytes);
  const int src_vec = src.Width(coefs);
  if (src_vec * value_bytes != h.sampleSize)
    Fail("Invalid HTK header in feature file: '" + name + "' mSampleSize do not match with parmKind");
  if (derivOrder < 0) derivOrder = src.order;
  trg.order = derivOrder;
  if (!Convertible(src, trg, h.sampleKind & 077, targetKind & 077))
    Fail("Cannot convert " + ParmKindStr(h.sampleKind) + " to " + ParmKindStr((unsigned)targetKind));
  const int kept_order = std::min(src.order, derivOrder);  // derivative blocks read from the file
  const int trg_vec = trg.Width(coefs);

  // the context frames come from the file's real neighbours where it has them; the rest is edge padding
  const int real_left = std::min(from_frame, cfg.startExt);
  const int real_right = std::min(h.nSamples - 1 - to_frame, cfg.endExt);
  from_frame -= real_left;
  to_frame += real_right;
  const int ext_left = cfg.startExt - real_left, ext_right = cfg.endExt - real_right;
  if (from_frame > to_frame || from_frame >= h.nSamples || to_frame < 0)
    Fail("Invalid frame range for feature file: '" + name + "'");
  const int tot = to_frame - from_frame + 1 + ext_left + ext_right;

  // the usual case -- float data whose source layout is the target's (same 0 / E / N flags, no derivative
  // dropped): the file's bytes go straight into the output rows, byte-swapped in place
  const bool direct = !comp && src.SameValues(trg, kept_order);
  out.rows = tot;
  out.cols = trg_vec;
  out.feats.resize((size_t)tot * trg_vec);  // a recycled buffer keeps its pages
  if (!direct) std::fill(out.feats.begin(), out.feats.end(), 0.0f);

  // the frames [from, to] in one read (the reference seeks and reads per frame, Features.cc:1207-1258)
  const int nread = to_frame - from_frame + 1;
  const size_t fbytes = (size_t)src_vec * value_bytes;
  const off_t first_byte = 12 + (comp ? (off_t)src_vec * 2 * 4 : 0) + (off_t)from_frame * (off_t)fbytes;
  // reads [first_byte + at, + bytes) into dst; a short file is the reference's per-frame read failure
  auto read_span = [&](char* dst, size_t at, size_t bytes) {
    for (size_t got = 0; got < bytes;) {
      const ssize_t r = pread(f.fd, dst + got, bytes - got, first_byte + (off_t)(at + got));
      if (r <= 0)
        Fail("Cannot read feature file: '" + name + "' frame " + std::to_string((at + got) / fbytes) + "/" +
             std::to_string(nread));
      got += (size_t)r;
    }
  };
  if (direct) {
    // 64-KiB pieces: each is byte-swapped while it is still in the core's cache after the read
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out.feats[(size_t)ext_left * trg_vec]);
    const size_t total = (size_t)nread * fbytes, piece = 64 * 1024;
    for (size_t done = 0; done < total; done += piece) {
      const size_t want = std::min(piece, total - done);  // a multiple of 4 bytes
      read_span(reinterpret_cast<char*>(dst) + done, done, want);
      if (cfg.swap)
        for (size_t k = done / 4; k < (done + want) / 4; k++) dst[k] = bswap32(dst[k]);
    }
  } else {
    thread_local std::vector<unsigned char> raw;
    raw.resize((size_t)nread * fbytes);
    read_span(reinterpret_cast<char*>(raw.data()), 0, raw.size());
    const std::vector<int> plan = src.PlacementIn(trg, coefs, kept_order);
    for (int r = 0; r < nread; r++) {
      const unsigned char* in = raw.data() + (size_t)r * fbytes;
      float* row = &out.feats[(size_t)(r + ext_left) * trg_vec];
      for (int si = 0; si < (int)plan.size(); si++) {  // the blocks read: the first kept_order + 1
        float v;
        if (comp) {  // int16 value x: (x + B) / A with the file's per-column scale A and bias B
          uint16_t x;
          memcpy(&x, in + 2 * si, 2);
          if (cfg.swap) x = bswap16(x);
          v = ((float)(int16_t)x + B[(size_t)si]) / A[(size_t)si];
        } else {
          uint32_t x;
          memcpy(&x, in + 4 * si, 4);
          if (cfg.swap) x = bswap32(x);
          memcpy(&v, &x, 4);
        }
        if (plan[(size_t)si] < trg_vec) row[plan[(size_t)si]] = v;
      }
    }
  }

  // the padding rows repeat the first / last real frame over the columns read from the file
  const int block = trg.Block(coefs);
  const size_t read_w = (size_t)(block * (1 + kept_order) - trg.suppressed);
  for (int i = 0; i < ext_left; i++)
    memcpy(&out.feats[(size_t)i * trg_vec], &out.feats[(size_t)ext_left * trg_vec], read_w * 4);
  for (int i = tot - ext_right; i < tot; i++)
    memcpy(&out.feats[(size_t)i * trg_vec], &out.feats[(size_t)(tot - ext_right - 1) * trg_vec], read_w * 4);

  float* M = out.feats.data();
  const size_t ld = (size_t)trg_vec;
  if (!cfg.cmn && !(kParmZ & h.sampleKind) && (kParmZ & targetKind)) {  // sentence mean (Features.cc:1279-1300)
    if (trg.suppressed)
      Fail("Cannot convert " + ParmKindStr(h.sampleKind) + " to " + ParmKindStr((unsigned)targetKind) +
           ": sentence mean normalisation with suppressed energy is not supported");
    for (int j = 0; j < block; j++) {
      float mean = 0.0f;
      for (int i = 0; i < tot; i++) mean += M[(size_t)i * ld + j];
      mean /= tot;
      for (int i = 0; i < tot; i++) M[(size_t)i * ld + j] -= mean;
    }
  }
  // derivative blocks the file does not have (Features.cc:1302-1343): regression over +-win frames, the
  // window shrunk to the frames that exist at the utterance's edges
  for (int order = src.order; order < derivOrder; order++) {
    if (trg.suppressed)
      Fail("Cannot convert " + ParmKindStr(h.sampleKind) + " to " + ParmKindStr((unsigned)targetKind) +
           ": derivatives of suppressed energy are not supported");
    const int win = order < (int)cfg.derivWin.size() ? cfg.derivWin[order] : 2;
    float norm = 0.0f;
    for (int k = 1; k <= win; k++) norm += 2 * k * k;
    const size_t from_col = (size_t)order * block, to_col = from_col + block;
    for (int i = 0; i < tot; i++) {
      const bool edge = i < win || i >= tot - win;
      for (int j = 0; j < block; j++) {
        const float* x = M + (size_t)i * ld + from_col + j;
        float acc = 0.0f;
        for (int k = 1; k <= win; k++) {
          const ptrdiff_t ahead = edge ? std::min(tot - 1 - i, k) : k, behind = edge ? std::min(i, k) : k;
          acc += k * (x[ahead * (ptrdiff_t)ld] - x[-behind * (ptrdiff_t)ld]);
        }
        M[(size_t)i * ld + to_col + j] = acc / norm;
      }
    }
  }

  if (cfg.cmn || cfg.cvn || cfg.cvg)
    ApplyCepsNorm(cfg, rec.logical, targetKind, derivOrder, block, trg.suppressed, trg_vec, tot, M);

  // CheckData's scan (the reference driver's, Matrix.h:238-252), done here on the reading thread
  out.bad_row = out.bad_col = -1;
  {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(out.feats.data());
    const size_t n = out.feats.size();
    uint32_t any = 0;
    for (size_t k = 0; k < n; k++) any |= (uint32_t)((w[k] & 0x7F800000u) == 0x7F800000u);
    if (any)
      for (size_t k = 0; k < n; k++)
        if ((w[k] & 0x7F800000u) == 0x7F800000u) {
          out.bad_row = (int)(k / (size_t)trg_vec);
          out.bad_col = (int)(k % (size_t)trg_vec);
          out.bad_value = out.feats[k];
          break;
        }
  }
  out.logical = rec.logical;
  out.samplePeriod = h.samplePeriod;
  // Features.cc:1345-1347 then 1383-1385: the derivative flags of the delivered order
  out.kind = (targetKind & ~(kParmD | kParmA | kParmT)) |
             (derivOrder == 3 ? (kParmD | kParmA | kParmT) : derivOrder == 2 ? (kParmD | kParmA) : derivOrder == 1 ? kParmD : 0);
}

std::string CheckDataError(const Utterance& u) {
  if (u.bad_row < 0) return std::string();
  std::ostringstream os;
  os << "Invalid value: " << u.bad_value << " in matrix row: " << u.bad_row << " col: " << u.bad_col
     << " file: " << u.logical;
  return os.str();
}

std::string MakeHtkFileName(const std::string& in, const char* outDir, const char* outExt) {
  if (in == "-") return "-";
  size_t slash = in.rfind('/');
  size_t base = slash == std::string::npos ? 0 : slash + 1;
  size_t bend = std::string::npos;
  if (outExt) bend = in.rfind('.');
  if (bend == std::string::npos || bend < base) bend = in.size();
  size_t dots = in.find("/./");
  if (dots != std::string::npos) base = dots + 3;
  std::string o;
  if (outDir) {
    if (*outDir) o += std::string(outDir) + "/";
    if (bend > base) o += in.substr(base, bend - base);
  } else {
    o += in.substr(0, bend);
  }
  if (outExt && *outExt) o += std::string(".") + outExt;
  return o;
}

// ------------------------------------------------------------------------------------------- MLF

namespace {
// A parameter-kind name as FeatureRepository::ReadParmKind(str, false) reads it (Features.cc:1438-1472):
// "_X" qualifiers peeled off the end, then the first base name that starts with what is left
int ParseKindName(const std::string& text) {
  static const char* const bases[13] = {"WAVEFORM", "LPC", "LPREFC", "LPCEPSTRA", "LPDELCEP", "IREFC", "MFCC",
                                        "FBANK", "MELSPEC", "USER", "DISCRETE", "PLP", "ANON"};
  static const std::pair<char, int> quals[] = {{'E', kParmE}, {'N', kParmN}, {'D', kParmD}, {'A', kParmA},
                                               {'C', kParmC}, {'Z', kParmZ}, {'K', 010000}, {'0', kParm0},
                                               {'V', 040000}, {'T', kParmT}};
  std::string base = text;
  int kind = 0;
  while (base.size() >= 2 && base[base.size() - 2] == '_') {
    const char q = base.back();
    const auto* it = std::find_if(std::begin(quals), std::end(quals), [q](const std::pair<char, int>& e) {
      return e.first == q;
    });
    if (it == std::end(quals)) return -1;
    kind |= it->second;
    base.resize(base.size() - 2);
  }
  for (int i = 0; i < 13; i++)
    if (std::string(bases[i]).compare(0, base.size(), base) == 0) return kind | i;
  return -1;
}

enum class NormFile { kMean, kVariance, kVarScale };

// The text of a normalisation file, read as a sequence of lexical items: "<...>" tags (1..64 characters
// other than '>'), integers, reals and whitespace-separated words (up to 64 characters shown).
class NormText {
 public:
  explicit NormText(const std::string& path) {
    std::ifstream in(path.c_str(), std::ios::binary);
    ok_ = in.good();
    if (ok_) text_.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
  }
  bool Opened() const { return ok_; }
  bool Tag(std::string* inner) {
    Blank();
    if (at_ >= text_.size() || text_[at_] != '<') return false;
    const size_t close = text_.find('>', at_ + 1);
    const size_t len = (close == std::string::npos ? text_.size() : close) - (at_ + 1);
    if (len == 0 || len > 64 || close == std::string::npos) return false;
    *inner = text_.substr(at_ + 1, len);
    at_ = close + 1;
    return true;
  }
  bool Int(int* v) {
    Blank();
    char* end = nullptr;
    const long x = strtol(text_.c_str() + at_, &end, 10);
    if (end == text_.c_str() + at_) return false;
    at_ = (size_t)(end - text_.c_str());
    *v = (int)x;
    return true;
  }
  bool Real(float* v) {
    Blank();
    char* end = nullptr;
    const float x = strtof(text_.c_str() + at_, &end);
    if (end == text_.c_str() + at_) return false;
    at_ = (size_t)(end - text_.c_str());
    *v = x;
    return true;
  }
  bool Word(std::string* w) {
    Blank();
    size_t e = at_;
    while (e < text_.size() && !isspace((unsigned char)text_[e])) e++;
    if (e == at_) return false;
    *w = text_.substr(at_, std::min<size_t>(e - at_, 64));
    at_ = e;
    return true;
  }

 private:
  void Blank() {
    while (at_ < text_.size() && isspace((unsigned char)text_[at_])) at_++;
  }
  std::string text_;
  size_t at_ = 0;
  bool ok_ = false;
};

std::string Upper(std::string s) {
  for (char& c : s) c = (char)toupper((unsigned char)c);
  return s;
}

// A CMN / CVN / VARSCALEFN file (FeatureRepository::ReadCepsNormFile, Features.cc:96-178): "<CEPSNORM> <kind>"
// (not in a VARSCALE file; the kind must be the features'), then "<MEAN|VARIANCE|VARSCALE> n" with n the
// expected count, n reals, nothing after them.  Tag names compare case-blind.  VARIANCE values are returned as
// 1 / sqrt(v), VARSCALE values as sqrt(v) (in double, as KaldiLib computes them).  The reference's error texts.
std::vector<float> ReadNormFile(const std::string& path, int sampleKind, NormFile type, int count,
                                const std::string& base = std::string()) {
  const char* section = type == NormFile::kMean ? "MEAN" : type == NormFile::kVariance ? "VARIANCE" : "VARSCALE";
  const char* what = type == NormFile::kMean ? "CMN" : type == NormFile::kVariance ? "CVN" : "VarScale";
  // a relative name opens against the creation-time directory; messages name the file as given
  NormText in(base.empty() || path.empty() || path[0] == '/' ? path : base + "/" + path);
  if (!in.Opened()) Fail(std::string("Cannot open ") + what + " pFileName: '" + path + "'");
  std::string tag, kind;
  bool header = true;
  if (type != NormFile::kVarScale)
    header = in.Tag(&tag) && in.Tag(&kind) && Upper(tag) == "CEPSNORM" && ParseKindName(kind) == sampleKind;
  int n = 0;
  header = header && in.Tag(&tag) && in.Int(&n) && Upper(tag) == section && n == count;
  if (!header) {
    const std::string prefix =
        type == NormFile::kVarScale ? std::string() : "<CEPSNORM> <" + ParmKindStr((unsigned)sampleKind) + ">";
    Fail(prefix + " <" + section + " ... expected in " + what + " file " + path);
  }
  std::vector<float> v((size_t)count);
  std::string word;
  for (float& x : v) {
    if (!in.Real(&x)) {
      if (in.Word(&word)) Fail("Decimal number expected but '" + word + "' found in " + what + " file " + path);
      Fail(std::string("Unexpected end of ") + what + " file " + path);
    }
    if (type == NormFile::kVariance) x = (float)(1 / sqrt((double)x));
    else if (type == NormFile::kVarScale) x = (float)sqrt((double)x);
  }
  if (in.Word(&word)) Fail("End of file expected but '" + word + "' found in " + what + " file " + path);
  return v;
}

// The normalisation file a mask picks for a logical name: the characters its '%'s capture ("" when it does not
// match), masks compiled once per thread
std::string MaskCapture(const std::string& logical, const std::string& mask) {
  thread_local std::unordered_map<std::string, LabelMask> compiled;
  auto it = compiled.find(mask);
  if (it == compiled.end()) it = compiled.emplace(mask, LabelMask::ForPath(mask)).first;
  std::string captured;
  it->second.Matches(LabelMask::AsPath(logical), &captured);
  return captured;
}
}  // namespace

void ApplyCepsNorm(const FeatureConfig& cfg, const std::string& logical, int targetKind, int derivOrder, int coefs,
                   int trg_N, int trg_vec, int tot, float* M) {
  // the parameter kind the files are checked against: mHeader.mSampleKind after the read (Features.cc:1349),
  // without _Z for the mean file, with the delivered derivative flags for the variance file (:1383-1385)
  int kind = targetKind & ~(kParmD | kParmA | kParmT);
  // the last file of each kind is kept (the reference re-reads only when the name changes)
  thread_local std::string last_cmn, last_cvn, last_cvg;  // (keyed with the base directory)
  thread_local std::vector<float> cmn, cvn, cvg;
  if (cfg.cmn) {
    std::string name = MaskCapture(logical, cfg.cmnMask);
    if (name.empty()) Fail("CMN Matching failed");
    name = (cfg.cmnDir.empty() ? std::string() : cfg.cmnDir + "/") + "/" + name;
    if (cfg.normBase + "|" + name != last_cmn) {
      last_cmn.clear();
      cmn = ReadNormFile(name, kind & ~kParmZ, NormFile::kMean, coefs, cfg.normBase);
      last_cmn = cfg.normBase + "|" + name;
    }
    for (int i = 0; i < tot; i++)
      for (int j = trg_N; j < coefs; j++) M[(size_t)i * trg_vec + (j - trg_N)] -= cmn[(size_t)j];
  }
  kind |= derivOrder == 3 ? (kParmD | kParmA | kParmT) : derivOrder == 2 ? (kParmD | kParmA) : derivOrder == 1 ? kParmD : 0;
  if (cfg.cvn) {
    std::string name = MaskCapture(logical, cfg.cvnMask);
    name = (cfg.cvnDir.empty() ? std::string() : cfg.cvnDir + "/") + "/" + name;
    if (cfg.normBase + "|" + name != last_cvn) {
      last_cvn.clear();
      cvn = ReadNormFile(name, kind, NormFile::kVariance, trg_vec, cfg.normBase);
      last_cvn = cfg.normBase + "|" + name;
    }
    for (int i = 0; i < tot; i++)
      for (int j = trg_N; j < trg_vec; j++) M[(size_t)i * trg_vec + (j - trg_N)] *= cvn[(size_t)j];
  }
  if (cfg.cvg) {
    if (cfg.normBase + "|" + cfg.cvgFile != last_cvg) {
      last_cvg.clear();
      cvg = ReadNormFile(cfg.cvgFile, -1, NormFile::kVarScale, trg_vec, cfg.normBase);
      last_cvg = cfg.normBase + "|" + cfg.cvgFile;
    }
    for (int i = 0; i < tot; i++)
      for (int j = trg_N; j < trg_vec; j++) M[(size_t)i * trg_vec + (j - trg_N)] *= cvg[(size_t)j];
  }
}

MlfLabels::MlfLabels(const std::string& mlf, const std::string& labelMap, const char* labelDir, const char* labelExt)
    : mMlf(mlf) {
  if (labelDir) mDirS = labelDir;
  if (labelExt) mExtS = labelExt;
  mDir = labelDir ? mDirS.c_str() : nullptr;
  mExt = labelExt ? mExtS.c_str() : nullptr;
  {  // ReadOutputLabelMap (Labels.cc:192-212)
    std::ifstream in(labelMap.c_str());
    if (!in.good()) Fail("Cannot open OutputLabelMapFile: " + labelMap);
    std::string tag;
    int i = 0;
    while (in >> tag) {
      if (mStates.count(tag)) Fail("Duplicate state tag: " + tag + " in " + labelMap);
      mStates[tag] = i++;
      mTags.push_back(tag);
    }
  }
  std::ifstream in(mlf.c_str());
  if (!in.good()) Fail("Cannot open Label MLF file: " + mlf);
  std::string line;
  Record* cur = nullptr;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (cur == nullptr) {
      std::string s = Trim(line);
      if (s.size() >= 2 && s[0] == '"') {
        size_t q = s.find('"', 1);
        std::string pat = s.substr(1, q == std::string::npos ? std::string::npos : q - 1);
        const size_t idx = mRecords.size();
        mRecords.emplace_back();
        cur = &mRecords.back();
        mIndex.Insert(pat, idx);
      }
      continue;
    }
    std::string s = Trim(line);
    if (s == ".") {
      cur = nullptr;
      continue;
    }
    if (s.empty() || s[0] == '#') continue;
    // GenDesiredMatrix's parse (Labels.cc:83-111): begin, end, state tag
    std::istringstream iss(s);
    Segment g;
    if (!(iss >> g.beg)) {
      if (cur->error.empty()) cur->error = "Cannot parse column 1 (begin)\nline: " + s;
      continue;
    }
    if (!(iss >> g.end)) {
      if (cur->error.empty()) cur->error = "Cannot parse column 2 (end)\nline: " + s;
      continue;
    }
    if (!(iss >> g.tag)) {
      if (cur->error.empty()) cur->error = "Cannot parse column 3 (state_tag)\nline: " + s;
      continue;
    }
    auto it = mStates.find(g.tag);
    g.state = it == mStates.end() ? -1 : it->second;
    cur->segs.push_back(g);
  }
}

size_t MlfLabels::ClassIds(const std::string& featureLogical, size_t nFrames, size_t sourceRate, int* out) const {
  const std::string lab = MakeHtkFileName(featureLogical, mDir, mExt);
  size_t found = 0;
  if (!mIndex.Find(lab, &found)) Fail("Cannot open label MLF record: " + lab);
  const Record* rec = &mRecords[found];
  if (nFrames < 1) Fail("Number of frames:" + std::to_string(nFrames) + " is lower than 1!!!\n" + featureLogical);
  if (!rec->error.empty()) Fail(rec->error + "\nfile: " + lab + "\n");
  if (sourceRate == 0) Fail("Zero sample period in features of " + featureLogical);
  std::fill(out, out + nFrames, -1);
  size_t trunc = 0;
  for (const Segment& g : rec->segs) {
    const unsigned long long beg = (g.beg + sourceRate / 2) / sourceRate;
    const unsigned long long end = (g.end + sourceRate / 2) / sourceRate;
    if (g.state < 0) Fail("Unknown state tag: '" + g.tag + "' file:'" + lab);
    for (unsigned long long t = beg; t < end; t++) {
      if (t >= nFrames) {
        trunc++;
        continue;
      }
      if (out[t] >= 0) {
        std::ostringstream os;
        os << "Frame already assigned to other state,  file: " << lab << " frame: " << t << " nframes: " << nFrames
           << " sum: 1 previously assigned to: " << mTags[(size_t)out[t]] << "(" << out[t] << ")"
           << " now should be assigned to: " << g.tag << "(" << g.state << ")\n";
        Fail(os.str());
      }
      out[t] = g.state;
    }
  }
  for (size_t t = 0; t < nFrames; t++)
    if (out[t] < 0) {
      std::ostringstream os;
      os << "Desired vector sum isn't 1.0,  file: " << lab << " row: " << t << " nframes: " << nFrames << "\n";
      Fail(os.str());
    }
  if (trunc > 10)
    std::cerr << "WARNING Truncated frames: " << trunc << " Check sourcerate in features and validity of labels"
              << std::endl;
  return trunc;
}

// ------------------------------------------------------------------------------------ read-ahead

FeatureReader::FeatureReader(const std::string& scp, const FeatureConfig& cfg, std::shared_ptr<const MlfLabels> labels,
                             int threads, int depth)
    : mCfg(cfg), mLabels(std::move(labels)), mThreads(std::max(1, threads)), mDepth(std::max(1, depth)) {
  std::ifstream in(scp.c_str());
  if (!in.good()) Fail("Cannot not open list file " + scp);
  // relative feature paths are taken from the working directory at creation (the reference's, which
  // reads them later from the same directory): the pool reads ahead, so a later chdir must not move them
  char cwd[4096];
  const std::string base = getcwd(cwd, sizeof(cwd)) ? std::string(cwd) : std::string();
  mCfg.normBase = base;  // the CMN / CVN files likewise
  std::string tok;
  while (in >> tok) {
    mRecords.push_back(ParseFileRecord(tok));
    mRecords.back().base = base;
  }
  mTargetKind = cfg.targetKind;
  mDerivOrder = cfg.derivOrder;
  if (!mRecords.empty()) {
    // the repository's latched target kind / derivative order come from the first file it reads
    try {
      HtkHeader h = ReadHtkHeader(mRecords[0].physical, cfg.swap, mRecords[0].base);
      unsigned kind = h.sampleKind & ~kParmC;
      if (mTargetKind == kParmAnon) {
        mTargetKind = (int)kind;
      } else if ((mTargetKind & 077) == kParmAnon) {
        mTargetKind = (mTargetKind & ~077) | (int)(kind & 077);
      }
      if (mDerivOrder < 0)
        mDerivOrder = (kind & kParmT) ? 3 : (kind & kParmA) ? 2 : (kind & kParmD) ? 1 : 0;
    } catch (std::exception& e) {
      mLatchError = e.what();
    }
  }
  Start();
}

FeatureReader::~FeatureReader() { Stop(); }

void FeatureReader::Start() {
  mStop = false;
  mIssued = mNext;
  for (int t = 0; t < mThreads; t++) mPool.emplace_back([this] { Worker(); });
}

void FeatureReader::Stop() {
  {
    std::lock_guard<std::mutex> g(mMu);
    mStop = true;
  }
  mCvWork.notify_all();
  for (auto& t : mPool) t.join();
  mPool.clear();
}

void FeatureReader::Worker() {
  for (;;) {
    size_t idx;
    {
      std::unique_lock<std::mutex> g(mMu);
      mCvWork.wait(g, [&] { return mStop || (mIssued < mRecords.size() && mIssued < mNext + (size_t)mDepth); });
      if (mStop) return;
      idx = mIssued++;
    }
    Slot s;
    try {
      if (!mLatchError.empty()) Fail(mLatchError);
      std::unique_ptr<Utterance> u;
      {
        std::lock_guard<std::mutex> g(mMu);
        if (!mFree.empty()) {
          u = std::move(mFree.back());
          mFree.pop_back();
        }
      }
      if (!u) u.reset(new Utterance);
      int tk = mTargetKind, dord = mDerivOrder;
      ReadHtkFeatures(mRecords[idx], mCfg, tk, dord, *u);
      if (mLabels) {  // targets of the trimmed rows (TNetCu.cc:390-401)
        const int rows = u->rows - mCfg.startExt - mCfg.endExt;
        if (rows < 1) Fail("Number of frames:" + std::to_string(rows) + " is lower than 1!!!\n" + u->logical);
        u->labels.resize((size_t)rows);
        mLabels->ClassIds(u->logical, (size_t)rows, (size_t)u->samplePeriod, u->labels.data());
      }
      s.u = std::move(u);
    } catch (std::exception& e) {
      s.error = e.what();
    }
    {
      std::lock_guard<std::mutex> g(mMu);
      mDone[idx] = std::move(s);
    }
    mCvDone.notify_all();
  }
}

const Utterance* FeatureReader::Next() {
  if (mCurrent) {  // its buffers serve a later record (no fresh pages per utterance)
    std::lock_guard<std::mutex> g(mMu);
    mFree.push_back(std::move(mCurrent));
  }
  if (mNext >= mRecords.size()) return nullptr;
  Slot s;
  {
    std::unique_lock<std::mutex> g(mMu);
    mCvDone.wait(g, [&] { return mDone.count(mNext) > 0; });
    s = std::move(mDone[mNext]);
    mDone.erase(mNext);
    mNext++;
  }
  mCvWork.notify_all();
  if (!s.error.empty()) Fail(s.error);
  mCurrent = std::move(s.u);
  return mCurrent.get();
}

void FeatureReader::Rewind() {
  Stop();
  mDone.clear();
  mCurrent.reset();
  mNext = 0;
  Start();
}

}  // namespace tnetio
