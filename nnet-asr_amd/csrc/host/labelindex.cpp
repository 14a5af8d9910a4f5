// labelindex.cpp -- label masks and the MLF record index (see labelindex.h for the behaviour followed).
#include "labelindex.h"

#include <algorithm>
#include <cstring>

namespace tnetio {

namespace {
// MlfStream.h's MAX_LABEL_DEPTH (PATH_MAX on Linux): the depth recorded for a name that is not "*"-led
constexpr size_t kWholeName = 4096;

bool IsSeparator(char c) { return c == '/' || c == '\\'; }
}  // namespace

// ------------------------------------------------------------------------------------------ LabelMask

LabelMask::LabelMask(const std::string& mask) : mMask(mask.c_str()) {  // C-string semantics: up to a NUL
  const size_t n = mMask.size();
  mNodes.resize(n + 1);
  for (size_t i = 0; i < n; i++) {
    Node& nd = mNodes[i];
    nd.ch = mMask[i];
    nd.set = -1;
    switch (mMask[i]) {
      case '*': nd.op = Op::kStar; break;
      case '?': nd.op = Op::kAny; break;
      case '%': nd.op = Op::kTake; mTakes++; break;
      case '[':
        nd.op = Op::kSet;
        nd.set = (int32_t)mSets.size();
        mSets.push_back(CompileSet(i));
        break;
      default: nd.op = Op::kChar;
    }
  }
  mNodes[n] = Node{Op::kEnd, '\0', -1};
}

// The member list of the set opening at `open`.  A member is a character or a range "lo-hi", either end
// possibly escaped with '\'; the list ends at an unescaped ']' that is not a range's upper end.  Reading
// stops at the first malformed member (an empty set, a range without an upper end, the mask ending inside
// the set).  Where a member holds, the set ends at the next unescaped ']' after that member.
LabelMask::Set LabelMask::CompileSet(size_t open) const {
  const std::string& m = mMask;  // m[m.size()] == '\0'
  auto close_from = [&m](size_t q) -> int32_t {
    for (; m[q] != ']'; q++) {
      if (m[q] == '\0') return -1;
      if (m[q] == '\\' && m[++q] == '\0') return -1;
    }
    return (int32_t)(q + 1);
  };
  Set s;
  size_t q = open + 1;
  if (m[q] == '!' || m[q] == '^') {
    s.negated = true;
    q++;
  }
  if (m[q] == ']') return s;  // "[]": malformed for every character
  while (m[q] != ']') {
    if (m[q] == '\\') q++;
    const char lo = m[q];
    if (lo == '\0') return s;
    char hi = lo;
    if (m[++q] == '-') {
      hi = m[++q];
      if (hi == '\0' || hi == ']') return s;
      if (hi == '\\' && (hi = m[++q]) == '\0') return s;
      q++;
    }
    s.members.push_back(Member{lo, hi, close_from(q)});
  }
  s.after = (int32_t)(q + 1);
  return s;
}

LabelMask::Result LabelMask::StepSet(const Set& s, char c, int32_t* next) const {
  for (const Member& mb : s.members)
    if (std::min(mb.lo, mb.hi) <= c && c <= std::max(mb.lo, mb.hi)) {
      if (s.negated) return Result::kMiss;
      if (mb.resume < 0) return Result::kBadSet;
      *next = mb.resume;
      return Result::kValid;
    }
  if (s.after < 0) return Result::kBadSet;  // no member held before the malformed one
  if (!s.negated) return Result::kMiss;
  *next = s.after;
  return Result::kValid;
}

// The program from node `pc` against the text from `t`.  `take` is where the next '%' writes its
// character (each write is NUL-terminated, the reference's capture buffer protocol).
LabelMask::Result LabelMask::Run(int32_t pc, const char* t, char* take) const {
  for (;; t++) {
    const Node& nd = mNodes[(size_t)pc];
    if (nd.op == Op::kEnd) return *t ? Result::kMiss : Result::kValid;
    if (*t == '\0')  // only a final lone '*' still matches an exhausted text
      return (nd.op == Op::kStar && mNodes[(size_t)pc + 1].op == Op::kEnd) ? Result::kValid : Result::kTextEnded;
    switch (nd.op) {
      case Op::kChar:
        if (*t != nd.ch) return Result::kMiss;
        pc++;
        break;
      case Op::kAny:
        pc++;
        break;
      case Op::kTake:
        *take++ = *t;
        *take = '\0';
        pc++;
        break;
      case Op::kSet: {
        const Result r = StepSet(mSets[(size_t)nd.set], *t, &pc);
        if (r != Result::kValid) return r;
        break;
      }
      case Op::kStar:
        return AfterStar(pc + 1, t, take);
      case Op::kEnd:
        break;
    }
  }
}

// A '*' at node pc - 1: the run of '?', '%' and '*' right after it consumes its characters first; then the
// star's extent grows one character at a time, trying the rest of the mask wherever its first character
// (or set) can start.  The search ends on a match, when the text runs out, or at a malformed set.
LabelMask::Result LabelMask::AfterStar(int32_t pc, const char* t, char* take) const {
  for (;; pc++) {
    const Op op = mNodes[(size_t)pc].op;
    if (op == Op::kStar) continue;
    if (op == Op::kAny) {
      if (*t++ == '\0') return Result::kTextEnded;
      continue;
    }
    if (op == Op::kTake) {
      *take++ = *t;
      *take = '\0';
      if (*t++ == '\0') return Result::kTextEnded;
      continue;
    }
    break;
  }
  const Node& lead = mNodes[(size_t)pc];
  if (lead.op == Op::kEnd) return Result::kValid;
  for (;; t++) {
    Result r = Result::kMiss;
    if (lead.op == Op::kSet || lead.ch == *t) r = Run(pc, t, take);
    if (*t == '\0') return Result::kTextEnded;
    if (r != Result::kMiss) return r;
  }
}

bool LabelMask::Matches(const std::string& text, std::string* captured) const {
  std::vector<char> buf(mTakes + 2, '\0');
  const bool ok = Run(0, text.c_str(), buf.data()) == Result::kValid;
  if (ok && captured) *captured = buf.data();
  return ok;
}

LabelMask LabelMask::ForPath(const std::string& mask) {
  return LabelMask(!mask.empty() && mask[0] == '*' ? mask : "*/" + mask);
}

std::string LabelMask::AsPath(const std::string& label) {
  return !label.empty() && label[0] == '/' ? label : "/" + label;
}

// ----------------------------------------------------------------------------------------- LabelIndex

void LabelIndex::Insert(const std::string& pattern, size_t rec) {
  if (!pattern.empty() && pattern[0] == '*')
    mDepths.insert((size_t)std::count_if(pattern.begin(), pattern.end(), IsSeparator));
  else
    mDepths.insert(kWholeName);
  if (pattern.find_first_of("*?%", 1) != std::string::npos) {
    mListed.emplace_back(LabelMask::ForPath(pattern), rec);
    return;
  }
  size_t covered;
  if (!Find(pattern, &covered)) mNamed[pattern] = Named{rec, mListed.size()};
}

bool LabelIndex::FindListed(const std::string& label, size_t first_n, size_t* rec) const {
  const std::string text = LabelMask::AsPath(label);
  const size_t n = first_n ? std::min(first_n, mListed.size()) : mListed.size();
  for (size_t k = 0; k < n; k++)
    if (mListed[k].first.Matches(text)) {
      *rec = mListed[k].second;
      return true;
    }
  return false;
}

// The hashed lookup.  The separators of the label, as positions, are walked by index: the first "*"-led
// depth d that the label has d separators for anchors the key at the d-th separator from the end, and each
// shallower depth moves the anchor towards the end by the difference.  Two properties of the reference's
// position arithmetic are kept: depth 0 (a "*name" pattern) anchors at the label's first character, and
// counting back past a separator at position 0 starts again from the last separator.
bool LabelIndex::FindNamed(const std::string& label, Named* hit) const {
  std::vector<size_t> seps;
  for (size_t i = 0; i < label.size(); i++)
    if (IsSeparator(label[i])) seps.push_back(i);
  auto probe = [&](const std::string& key) {
    auto it = mNamed.find(key);
    if (it == mNamed.end()) return false;
    *hit = it->second;
    return true;
  };
  bool anchored = false;
  size_t anchor = 0, anchor_depth = 0;  // anchor: index into seps (depth 0: the label's start)
  for (const size_t d : mDepths) {
    if (d == kWholeName) {
      if (probe(label)) return true;
      continue;
    }
    if (!anchored) {
      if (d == 0) {
        anchored = true;
        anchor_depth = 0;
        if (probe("*" + label)) return true;
        continue;
      }
      size_t left = seps.size(), idx = 0;
      bool ok = true;
      for (size_t step = 0; step < d; step++) {
        if (left == 0) {
          ok = false;
          break;
        }
        idx = --left;
        if (seps[idx] == 0) left = seps.size();
      }
      if (!ok) continue;  // too few separators for this depth: the next one starts afresh
      anchored = true;
      anchor = idx;
      anchor_depth = d;
    } else {
      anchor += anchor_depth - d;
      anchor_depth = d;
      if (anchor >= seps.size()) return false;
    }
    if (probe("*" + label.substr(seps[anchor]))) return true;
  }
  return false;
}

bool LabelIndex::Find(const std::string& label, size_t* rec) const {
  Named hit;
  if (FindNamed(label, &hit)) {
    *rec = hit.rec;
    FindListed(label, hit.listed, rec);  // an earlier pattern wins
    return true;
  }
  return FindListed(label, 0, rec);
}

}  // namespace tnetio
