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

  int src_deriv = (h.sampleKind & kParmT) ? 3 : (h.sampleKind & kParmA) ? 2 : (h.sampleKind & kParmD) ? 1 : 0;
  const int src_E = (h.sampleKind & kParmE) != 0;
  const int src_0 = (h.sampleKind & kParm0) != 0;
  const int src_N = ((h.sampleKind & kParmN) != 0) * (src_E + src_0);
  h.sampleKind &= ~kParmC;
  if (targetKind == kParmAnon) {
    targetKind = h.sampleKind;
  } else if ((targetKind & 077) == kParmAnon) {
    targetKind &= ~077;
    targetKind |= h.sampleKind & 077;
  }
  const int trg_E = (targetKind & kParmE) != 0;
  const int trg_0 = (targetKind & kParm0) != 0;
  const int trg_N = ((targetKind & kParmN) != 0) * (trg_E + trg_0);

  const int coef_size = comp ? 2 : 4;
  int coefs = (h.sampleSize / coef_size + src_N) / (src_deriv + 1) - src_E - src_0;
  const int src_vec = (coefs + src_E + src_0) * (src_deriv + 1) - src_N;
  if (src_vec * coef_size != h.sampleSize)
    Fail("Invalid HTK header in feature file: '" + name + "' mSampleSize do not match with parmKind");
  if (derivOrder < 0) derivOrder = src_deriv;

  if ((!src_E && trg_E) || (!src_0 && trg_0) || (src_N && !trg_N) || (trg_N && !trg_E && !trg_0) ||
      (trg_N && !derivOrder) || (src_N && !src_deriv && derivOrder) ||
      ((h.sampleKind & 077) != (targetKind & 077) && (h.sampleKind & 077) != kParmAnon))
    Fail("Cannot convert " + ParmKindStr(h.sampleKind) + " to " + ParmKindStr((unsigned)targetKind));

  const int lo_deriv = std::min(src_deriv, derivOrder);
  const int trg_vec = (coefs + trg_E + trg_0) * (derivOrder + 1) - trg_N;

  int ext_left = cfg.startExt, ext_right = cfg.endExt;
  int i = std::min(from_frame, cfg.startExt);
  from_frame -= i;
  ext_left -= i;
  i = std::min(h.nSamples - to_frame - 1, cfg.endExt);
  to_frame += i;
  ext_right -= i;
  if (from_frame > to_frame || from_frame >= h.nSamples || to_frame < 0)
    Fail("Invalid frame range for feature file: '" + name + "'");
  const int tot = to_frame - from_frame + 1 + ext_left + ext_right;

  out.rows = tot;
  out.cols = trg_vec;
  out.feats.resize((size_t)tot * trg_vec);  // every element is written below (a recycled buffer keeps its pages)
  if (!(!comp && src_vec == trg_vec))
    std::fill(out.feats.begin(), out.feats.end(), 0.0f);

  // the frames [from, to] in one read (the reference seeks and reads per frame, Features.cc:1207-1258)
  const int nread = to_frame - from_frame + 1;
  const size_t fbytes = (size_t)src_vec * coef_size;
  const off_t base = 12 + (comp ? (off_t)src_vec * 2 * 4 : 0) + (off_t)from_frame * (off_t)fbytes;
  auto read_block = [&](void* dst, size_t bytes) {  // a short file is the reference's per-frame read failure
    char* p = static_cast<char*>(dst);
    size_t n = bytes;
    off_t off = base;
    while (n) {
      ssize_t r = pread(f.fd, p, n, off);
      if (r <= 0) Fail("Cannot read feature file: '" + name + "' frame " + std::to_string((bytes - n) / fbytes) + "/" +
                       std::to_string(nread));
      p += r;
      n -= (size_t)r;
      off += r;
    }
  };
  // the usual case -- float data whose source layout is the target's (same 0 / E / N flags, no derivative
  // dropped): straight into the output rows, byte-swapped in place
  const bool direct = !comp && src_vec == trg_vec && lo_deriv == src_deriv && src_E == trg_E && src_0 == trg_0 &&
                      src_N == trg_N;
  if (direct) {
    // 64-KiB pieces: each is byte-swapped while it is still in the core's cache after the read
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out.feats[(size_t)ext_left * trg_vec]);
    const size_t total = (size_t)nread * fbytes;
    const size_t piece = 64 * 1024;
    char* p = reinterpret_cast<char*>(dst);
    for (size_t done = 0; done < total;) {
      const size_t want = std::min(piece, total - done);  // a multiple of 4 bytes
      for (size_t got = 0; got < want;) {
        ssize_t r = pread(f.fd, p + done + got, want - got, base + (off_t)(done + got));
        if (r <= 0) Fail("Cannot read feature file: '" + name + "' frame " + std::to_string((done + got) / fbytes) +
                         "/" + std::to_string(nread));
        got += (size_t)r;
      }
      if (cfg.swap)
        for (size_t k = done / 4; k < (done + want) / 4; k++) dst[k] = bswap32(dst[k]);
      done += want;
    }
  } else {
    thread_local std::vector<unsigned char> raw;
    raw.resize((size_t)nread * fbytes);
    read_block(raw.data(), raw.size());
    // decode one source frame into the target layout (the reads of Features.cc:1223-1246, including
    // their overwrite of a source 0 / E value the target does not keep); `tmp` has room past the row
    std::vector<float> tmp((size_t)trg_vec + 8);
    for (int r = 0; r < nread; r++) {
      const unsigned char* src = raw.data() + (size_t)r * fbytes;
      int si = 0;  // next source value
      const float* Ap = A.data();
      const float* Bp = B.data();
      auto read = [&](float* dst, int n) {
        for (int k = 0; k < n; k++, si++) {
          if (comp) {
            uint16_t v;
            memcpy(&v, src + 2 * si, 2);
            if (cfg.swap) v = bswap16(v);
            dst[k] = ((float)(int16_t)v + Bp[k]) / Ap[k];
          } else {
            uint32_t v;
            memcpy(&v, src + 4 * si, 4);
            if (cfg.swap) v = bswap32(v);
            memcpy(&dst[k], &v, 4);
          }
        }
        Ap += n;
        Bp += n;
      };
      float* mx = tmp.data();
      read(mx, coefs);
      mx += coefs;
      if (src_0 && !src_N) read(mx, 1);
      if (trg_0 && !trg_N) mx++;
      if (src_E && !src_N) read(mx, 1);
      if (trg_E && !trg_N) mx++;
      for (int j = 0; j < lo_deriv; j++) {
        read(mx, coefs);
        mx += coefs;
        if (src_0) read(mx, 1);
        if (trg_0) mx++;
        if (src_E) read(mx, 1);
        if (trg_E) mx++;
      }
      memcpy(&out.feats[(size_t)(r + ext_left) * trg_vec], tmp.data(), (size_t)trg_vec * 4);
      std::fill(tmp.begin(), tmp.end(), 0.0f);
    }
  }

  coefs += trg_0 + trg_E;
  const size_t ext_w = (size_t)(coefs * (1 + lo_deriv) - trg_N);
  for (i = 0; i < ext_left; i++)
    memcpy(&out.feats[(size_t)i * trg_vec], &out.feats[(size_t)ext_left * trg_vec], ext_w * 4);
  for (i = tot - ext_right; i < tot; i++)
    memcpy(&out.feats[(size_t)i * trg_vec], &out.feats[(size_t)(tot - ext_right - 1) * trg_vec], ext_w * 4);

  float* M = out.feats.data();
  if (!cfg.cmn && !(kParmZ & h.sampleKind) && (kParmZ & targetKind)) {  // sentence mean (Features.cc:1279-1300)
    if (trg_N) Fail("Cannot convert " + ParmKindStr(h.sampleKind) + " to " + ParmKindStr((unsigned)targetKind) +
                    ": sentence mean normalisation with suppressed energy is not supported");
    for (int j = 0; j < coefs; j++) {
      float norm = 0.0f;
      for (i = 0; i < tot; i++) norm += M[(size_t)i * trg_vec + j];
      norm /= tot;
      for (i = 0; i < tot; i++) M[(size_t)i * trg_vec + j] -= norm;
    }
  }
  for (; src_deriv < derivOrder; src_deriv++) {  // missing derivatives (Features.cc:1302-1343)
    if (trg_N) Fail("Cannot convert " + ParmKindStr(h.sampleKind) + " to " + ParmKindStr((unsigned)targetKind) +
                    ": derivatives of suppressed energy are not supported");
    const int win = src_deriv < (int)cfg.derivWin.size() ? cfg.derivWin[src_deriv] : 2;
    float norm = 0.0f;
    for (int k = 1; k <= win; k++) norm += 2 * k * k;
    for (i = 0; i < tot; i++)
      for (int j = 0; j < coefs; j++) {
        const float* s = M + (size_t)i * trg_vec + (size_t)src_deriv * coefs + j;
        float d = 0.0f;
        for (int k = 1; k <= win; k++) {
          const int up = (i < win || i >= tot - win) ? std::min(tot - 1 - i, k) : k;
          const int dn = (i < win || i >= tot - win) ? std::min(i, k) : k;
          d += k * (s[(ptrdiff_t)up * trg_vec] - s[-(ptrdiff_t)dn * trg_vec]);
        }
        M[(size_t)i * trg_vec + (size_t)src_deriv * coefs + j + coefs] = d / norm;
      }
  }

  if (cfg.cmn || cfg.cvn || cfg.cvg) ApplyCepsNorm(cfg, rec.logical, targetKind, derivOrder, coefs, trg_N, trg_vec, tot, M);

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
// The STK wildcard matcher the reference's MLF lookup uses (KaldiLib/StkMatch.cc matche /
// matche_after_star): '?' and '%' one character, '*' any run, [..] / [!..] / [^..] sets with ranges and
// backslash escapes inside a set, a text that ends early matches only a trailing '*'.  Restated step for
// step (the return codes steer matche_after_star's search); parity: tests/test_reader.py MLF cases.
enum { kMatchValid = 1, kMatchEnd, kMatchAbort, kMatchRange, kMatchLiteral, kMatchPattern };
int StkMatchAfterStar(const char* p, const char* t, char* s);
int StkMatche(const char* p, const char* t, char* s) {
  for (; *p; p++, t++) {
    if (!*t) return (*p == '*' && *++p == '\0') ? kMatchValid : kMatchAbort;
    switch (*p) {
      case '?':
        break;
      case '%':  // one character, captured
        *s++ = *t;
        *s = '\0';
        break;
      case '*':
        return StkMatchAfterStar(p, t, s);
      case '[': {
        p++;
        bool invert = false;
        if (*p == '!' || *p == '^') {
          invert = true;
          p++;
        }
        if (*p == ']') return kMatchPattern;
        bool member = false, loop = true;
        while (loop) {
          if (*p == ']') {
            loop = false;
            continue;
          }
          char lo, hi;
          if (*p == '\\') lo = hi = *++p;
          else lo = hi = *p;
          if (!*p) return kMatchPattern;
          if (*++p == '-') {
            hi = *++p;
            if (hi == '\0' || hi == ']') return kMatchPattern;
            if (hi == '\\') {
              hi = *++p;
              if (!hi) return kMatchPattern;
            }
            p++;
          }
          if (lo < hi) {
            if (*t >= lo && *t <= hi) member = true, loop = false;
          } else if (*t >= hi && *t <= lo) {
            member = true, loop = false;
          }
        }
        if ((invert && member) || !(invert || member)) return kMatchRange;
        if (member) {
          while (*p != ']') {
            if (!*p) return kMatchPattern;
            if (*p == '\\') {
              p++;
              if (!*p) return kMatchPattern;
            }
            p++;
          }
        }
        break;
      }
      default:
        if (*p != *t) return kMatchLiteral;
    }
  }
  return *t ? kMatchEnd : kMatchValid;
}
int StkMatchAfterStar(const char* p, const char* t, char* s) {
  int match = 0;
  while (*p == '?' || *p == '%' || *p == '*') {
    if (*p == '?' && !*t++) return kMatchAbort;
    if (*p == '%') {
      *s++ = *t;
      *s = '\0';
      if (!*t++) return kMatchAbort;
    }
    p++;
  }
  if (!*p) return kMatchValid;
  const char nextp = *p;
  do {
    if (nextp == *t || nextp == '[') match = StkMatche(p, t, s);
    if (!*t++) match = kMatchAbort;
  } while (match != kMatchValid && match != kMatchAbort && match != kMatchPattern);
  return match;
}
// ProcessMask (StkMatch.cc:453-490) as LabelContainer::FindInList calls it: "*/" prepended to a pattern that
// does not start with '*', "/" to a label that does not start with '/'
// (with the characters the '%'s capture: the CMN / CVN file names, Features.cc:1359-1392)
bool ProcessMask(const std::string& label, const std::string& pattern, std::string* captured) {
  std::vector<char> sub((size_t)std::count(pattern.begin(), pattern.end(), '%') + 2, '\0');
  const std::string w = (pattern.empty() || pattern[0] != '*') ? "*/" + pattern : pattern;
  const std::string t = (label.empty() || label[0] != '/') ? "/" + label : label;
  const bool ok = StkMatche(w.c_str(), t.c_str(), sub.data()) == kMatchValid;
  if (captured) *captured = ok ? std::string(sub.data()) : std::string();
  return ok;
}
bool MaskMatches(const std::string& label, const std::string& pattern) { return ProcessMask(label, pattern, nullptr); }

// FeatureRepository::ReadParmKind(str, false) (Features.cc:1438-1472), its prefix match of the base name included
int ReadParmKindRef(const char* str) {
  static const char* names[13] = {"WAVEFORM", "LPC", "LPREFC", "LPCEPSTRA", "LPDELCEP", "IREFC", "MFCC",
                                  "FBANK", "MELSPEC", "USER", "DISCRETE", "PLP", "ANON"};
  int kind = 0;
  int slen = (int)strlen(str);
  for (; slen >= 2 && str[slen - 2] == '_'; slen -= 2) {
    const char q = str[slen - 1];
    kind |= q == 'E' ? kParmE : q == 'N' ? kParmN : q == 'D' ? kParmD : q == 'A' ? kParmA : q == 'C' ? kParmC
          : q == 'Z' ? kParmZ : q == 'K' ? 010000 : q == '0' ? kParm0 : q == 'V' ? 040000 : q == 'T' ? kParmT : -1;
    if (kind == -1) return -1;
  }
  for (int i = 0; i < 13; i++)
    if (!strncmp(str, names[i], (size_t)slen)) return kind | i;
  return -1;
}

enum CepsNormType { kCnfMean, kCnfVariance, kCnfVarScale };

// FeatureRepository::ReadCepsNormFile (Features.cc:96-178), the same stdio parse and error texts: a header
// "<CEPSNORM> <kind>" (not for VARSCALE), "<MEAN|VARIANCE|VARSCALE> n" with n == coefs, n numbers, end of file;
// VARIANCE values become 1 / sqrt(v), VARSCALE values sqrt(v)
std::vector<float> ReadCepsNormFile(const std::string& name, int sampleKind, CepsNormType type, int coefs) {
  const char* typeStr = type == kCnfMean ? "MEAN" : type == kCnfVariance ? "VARIANCE" : "VARSCALE";
  const char* typeStr2 = type == kCnfMean ? "CMN" : type == kCnfVariance ? "CVN" : "VarScale";
  FILE* fp = fopen(name.c_str(), "r");
  if (!fp) Fail(std::string("Cannot open ") + typeStr2 + " pFileName: '" + name + "'");
  struct Closer {
    FILE* f;
    ~Closer() { fclose(f); }
  } closer{fp};
  char s1[80] = {0}, s2[80] = {0};
  int n = 0;
  auto up = [](char* c) {
    for (char* q = c; *q; q++) *q = (char)toupper((unsigned char)*q);
    return c;
  };
  if ((type != kCnfVarScale && (fscanf(fp, " <%64[^>]> <%64[^>]>", s1, s2) != 2 || strcmp(up(s1), "CEPSNORM") ||
                                ReadParmKindRef(s2) != sampleKind)) ||
      fscanf(fp, " <%64[^>]> %d", s1, &n) != 2 || strcmp(up(s1), typeStr) || n != coefs) {
    const std::string k = ParmKindStr((unsigned)sampleKind);
    Fail(std::string("") + (type == kCnfVarScale ? "" : "<CEPSNORM> <") + (type == kCnfVarScale ? "" : k) +
         (type == kCnfVarScale ? "" : ">") + " <" + typeStr + " ... expected in " + typeStr2 + " file " + name);
  }
  std::vector<float> v((size_t)coefs);
  for (int i = 0; i < coefs; i++) {
    if (fscanf(fp, " %g", &v[(size_t)i]) != 1) {
      if (fscanf(fp, "%64s", s2) == 1)
        Fail(std::string("Decimal number expected but '") + s2 + "' found in " + typeStr2 + " file " + name);
      else if (feof(fp))
        Fail(std::string("Unexpected end of ") + typeStr2 + " file " + name);
      else
        Fail(std::string("Cannot read ") + typeStr2 + " file " + name);
    }
    // double arithmetic: KaldiLib calls the C library's sqrt(double) (measured bit-exact against the reference)
    if (type == kCnfVariance) v[(size_t)i] = (float)(1 / sqrt((double)v[(size_t)i]));
    else if (type == kCnfVarScale) v[(size_t)i] = (float)sqrt((double)v[(size_t)i]);
  }
  if (fscanf(fp, "%64s", s2) == 1)
    Fail(std::string("End of file expected but '") + s2 + "' found in " + typeStr2 + " file " + name);
  return v;
}
}  // namespace

void ApplyCepsNorm(const FeatureConfig& cfg, const std::string& logical, int targetKind, int derivOrder, int coefs,
                   int trg_N, int trg_vec, int tot, float* M) {
  // the parameter kind the files are checked against: mHeader.mSampleKind after the read (Features.cc:1349),
  // without _Z for the mean file, with the delivered derivative flags for the variance file (:1383-1385)
  int kind = targetKind & ~(kParmD | kParmA | kParmT);
  // the last file of each kind is kept (the reference re-reads only when the name changes)
  thread_local std::string last_cmn, last_cvn, last_cvg;
  thread_local std::vector<float> cmn, cvn, cvg;
  if (cfg.cmn) {
    std::string name;
    ProcessMask(logical, cfg.cmnMask, &name);
    if (name.empty()) Fail("CMN Matching failed");
    name = (cfg.cmnDir.empty() ? std::string() : cfg.cmnDir + "/") + "/" + name;
    if (name != last_cmn) {
      last_cmn.clear();
      cmn = ReadCepsNormFile(name, kind & ~kParmZ, kCnfMean, coefs);
      last_cmn = name;
    }
    for (int i = 0; i < tot; i++)
      for (int j = trg_N; j < coefs; j++) M[(size_t)i * trg_vec + (j - trg_N)] -= cmn[(size_t)j];
  }
  kind |= derivOrder == 3 ? (kParmD | kParmA | kParmT) : derivOrder == 2 ? (kParmD | kParmA) : derivOrder == 1 ? kParmD : 0;
  if (cfg.cvn) {
    std::string name;
    ProcessMask(logical, cfg.cvnMask, &name);
    name = (cfg.cvnDir.empty() ? std::string() : cfg.cvnDir + "/") + "/" + name;
    if (name != last_cvn) {
      last_cvn.clear();
      cvn = ReadCepsNormFile(name, kind, kCnfVariance, trg_vec);
      last_cvn = name;
    }
    for (int i = 0; i < tot; i++)
      for (int j = trg_N; j < trg_vec; j++) M[(size_t)i * trg_vec + (j - trg_N)] *= cvn[(size_t)j];
  }
  if (cfg.cvg) {
    if (cfg.cvgFile != last_cvg) {
      last_cvg.clear();
      cvg = ReadCepsNormFile(cfg.cvgFile, -1, kCnfVarScale, trg_vec);
      last_cvg = cfg.cvgFile;
    }
    for (int i = 0; i < tot; i++)
      for (int j = trg_N; j < trg_vec; j++) M[(size_t)i * trg_vec + (j - trg_N)] *= cvg[(size_t)j];
  }
}

namespace {
// PATH_MAX on Linux: MlfStream.h's MAX_LABEL_DEPTH, the depth of a name without a leading '*'
constexpr size_t kMaxLabelDepth = 4096;
size_t DirDepth(const std::string& path) {
  return (size_t)std::count(path.begin(), path.end(), '/') + (size_t)std::count(path.begin(), path.end(), '\\');
}
}  // namespace

// LabelContainer::FindInHash (MlfStream.cc:97-197), the reference's position arithmetic kept as it is
// (including find_last_of from prev - 1 when prev is 0, which wraps to the whole label)
bool MlfLabels::FindInHash(const std::string& label, size_t* rec, size_t* limit) const {
  bool found = false;
  std::string str;
  size_t current_depth = kMaxLabelDepth, prev = label.size() + 1;
  auto lookup = [&](const std::string& key) {
    auto it = mHash.find(key);
    if (it == mHash.end()) return false;
    *rec = it->second.rec;
    *limit = it->second.limit;
    return true;
  };
  for (auto ri = mDepths.rbegin(); !found && ri != mDepths.rend(); ++ri) {
    if (*ri == kMaxLabelDepth) {
      found = lookup(label);
    } else if (current_depth == kMaxLabelDepth) {
      if (*ri > 0) {
        for (size_t i = 1; i <= *ri && prev != std::string::npos; i++) prev = label.find_last_of("/\\", prev - 1);
      } else {
        prev = 0;
      }
      if (prev != std::string::npos) {
        str.assign(label, prev, label.size());
        str = '*' + str;
        found = lookup(str);
        current_depth = *ri;
      } else {
        prev = label.size() + 1;
      }
    } else {
      while (current_depth > *ri) {
        if ((prev = label.find_first_of("/\\", prev + 1)) != std::string::npos) current_depth--;
        else return false;
      }
      str.assign(label, prev, label.size());
      str = '*' + str;
      found = lookup(str);
    }
  }
  return found;
}

// LabelContainer::FindInList (MlfStream.cc:201-239): the first of the first `limit` patterns (0: all) that
// ProcessMask matches
bool MlfLabels::FindInList(const std::string& label, size_t limit, size_t* rec) const {
  const size_t n = limit ? std::min(limit, mList.size()) : mList.size();
  for (size_t k = 0; k < n; k++)
    if (MaskMatches(label, mList[k].first)) {
      *rec = mList[k].second;
      return true;
    }
  return false;
}

// LabelContainer::Find (MlfStream.cc:243-262): a hash hit can be overridden by a list pattern defined before it
const MlfLabels::Record* MlfLabels::Find(const std::string& label) const {
  size_t rec = 0, limit = 0;
  if (FindInHash(label, &rec, &limit)) {
    (void)FindInList(label, limit, &rec);
    return &mRecords[rec];
  }
  return FindInList(label, 0, &rec) ? &mRecords[rec] : nullptr;
}

// LabelContainer::Insert (MlfStream.cc:43-93): a pattern with no wildcard after its first character is
// hashed -- unless an earlier definition (hashed or listed) already matches it -- else listed; every
// '*'-led pattern records its directory depth for FindInHash's walk
void MlfLabels::Insert(const std::string& pattern, size_t rec) {
  mDepths.insert(!pattern.empty() && pattern[0] == '*' ? DirDepth(pattern) : kMaxLabelDepth);
  if (pattern.find_first_of("*?%", 1) == std::string::npos) {
    if (!Find(pattern)) mHash[pattern] = Hashed{rec, mList.size()};
  } else {
    mList.emplace_back(pattern, rec);
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
        Insert(pat, idx);
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
  const Record* rec = Find(lab);
  if (!rec) Fail("Cannot open label MLF record: " + lab);
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
