// htkio.h -- the host front end of the TNetCu intake: HTK feature files, the script list and the
// master label file, read natively and ahead of the trainer by a pool of reader threads.
//
// Reference:
//   FileListElem            src/KaldiLib/Features.cc:41-83    "logical=physical[s,e]{weight}" records
//   FeatureRepository::ReadHTKFeatures  Features.cc:1009-1347  header, parameter kinds, compressed form,
//                                                             frame range, STARTFRMEXT/ENDFRMEXT edge
//                                                             replication, sentence mean (_Z), deltas
//   LabelRepository::GenDesiredMatrix   src/KaldiLib/Labels.cc:42-186  MLF segments -> per-frame targets
//   LabelContainer::Find                src/KaldiLib/MlfStream.cc:96-265  "*/name.lab" pattern lookup (labelindex.h)
//   MakeHtkFileName                     src/KaldiLib/Common.cc:118-172
// The reference reads a file frame by frame (an fseek + fread per frame, Features.cc:1207-1258) on the
// training thread, between cache fills (TNetCu.cc:376-419).  Here a file is one pread into memory,
// decoded (byte order, int16 decompression) in place, and up to `depth` utterances are read ahead of
// the consumer by `threads` workers, delivered strictly in script order.  Targets come out as class
// ids (one int per frame) -- the one-hot rows of GenDesiredMatrix, as the trainer consumes them.
//   CMN / CVN / VARSCALEFN              Features.cc:96-178, 1350-1410  normalisation files by mask
#pragma once

#include <condition_variable>
#include <cstdint>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "labelindex.h"

namespace tnetio {

// HTK parameter kinds (src/KaldiLib/Features.h:46-69)
enum : int {
  kParmAnon = 12,
  kParmE = 0000100,
  kParmN = 0000200,
  kParmD = 0000400,
  kParmA = 0001000,
  kParmC = 0002000,
  kParmZ = 0004000,
  kParm0 = 0020000,
  kParmT = 0100000,
};

struct HtkHeader {
  int32_t nSamples = 0;
  int32_t samplePeriod = 0;
  int16_t sampleSize = 0;
  uint16_t sampleKind = 0;
};

// one script line (FileListElem, Features.cc:41-83)
struct FileRecord {
  std::string logical, physical;
  float weight = 1.0f;
  std::string base;  // directory relative physical names are opened from ("" = the current one)
};
FileRecord ParseFileRecord(const std::string& line);

struct FeatureConfig {
  bool swap = true;          // !NATURALREADORDER on a little-endian host (TNetCu.cc:192)
  int startExt = 0, endExt = 0;
  int targetKind = kParmAnon;  // TARGETKIND (UserInterface.cc:411-417); ANON latches the first file's kind
  int derivOrder = 0;        // 0 with TARGETKIND=ANON (UserInterface.cc:444-459); < 0: the first file's
  std::vector<int> derivWin; // DELTAWINDOW / ACCWINDOW / THIRDWINDOW (default 2 each)
  // cepstral mean / variance normalisation files (UserInterface.cc:385-410, Features.cc:1352-1410): active when
  // the mask is set; the file is <dir>/ + "/" + the characters the mask's '%'s capture from the logical name
  bool cmn = false, cvn = false, cvg = false;
  std::string cmnDir, cmnMask;  // CMEANDIR, CMEANMASK
  std::string cvnDir, cvnMask;  // VARSCALEDIR, VARSCALEMASK
  std::string cvgFile;          // VARSCALEFN
  // the working directory at the reader's creation: relative normalisation files are opened against it (the pool
  // reads ahead, so a later chdir must not move them), and named as given in every message
  std::string normBase;
};

struct Utterance {
  std::string logical;
  std::vector<float> feats;  // rows x cols, row-major, dense
  int rows = 0, cols = 0;
  int samplePeriod = 0;      // of the file (GenDesiredMatrix's sourceRate)
  int kind = 0;              // the matrix's parameter kind (mHeader.mSampleKind after the read)
  std::vector<int> labels;   // class ids of rows - startExt - endExt frames (empty without labels)
  // the first NaN / Inf of the matrix in row-major order (bad_row < 0: none) -- what TNetCu's
  // feats_host.CheckData (TNetCu.cc:386, Matrix.h:238-252) rejects; found by the reading thread
  int bad_row = -1, bad_col = -1;
  float bad_value = 0.0f;
};

// TNetCu's CheckData message for u's first invalid value ("" if none)
std::string CheckDataError(const Utterance& u);

// Reads one record into `out` (feats, rows, cols, samplePeriod, kind).  `targetKind` / `derivOrder`
// are the repository's latched state (ANON / < 0 resolve to this file's).  Throws std::runtime_error
// with the reference's messages.
void ReadHtkFeatures(const FileRecord& rec, const FeatureConfig& cfg, int& targetKind, int& derivOrder,
                     Utterance& out);

// Header of a record's physical file (frame-range suffix ignored), byte order as configured.
HtkHeader ReadHtkHeader(const std::string& physical, bool swap, const std::string& base = std::string());

// MakeHtkFileName (Common.cc:118-172)
std::string MakeHtkFileName(const std::string& in, const char* outDir, const char* outExt);

// LabelRepository: the MLF indexed once (pattern -> its segment lines), the state-tag map
// (ReadOutputLabelMap, Labels.cc:192-212).  Lookups are const and thread-safe.
class MlfLabels {
 public:
  MlfLabels(const std::string& mlf, const std::string& labelMap, const char* labelDir, const char* labelExt);
  // GenDesiredMatrix as class ids: out[t] = the state of frame t.  Errors as the reference: unknown
  // tag, a frame assigned twice, a frame never assigned (the row-sum check); frames past nFrames are
  // dropped and counted (> 10: the reference's "Truncated frames" warning).  Returns that count.
  size_t ClassIds(const std::string& featureLogical, size_t nFrames, size_t sourceRate, int* out) const;
  size_t NumStates() const { return mStates.size(); }

 private:
  struct Segment {
    unsigned long long beg, end;
    int state;        // -1: unknown tag (an error only when the record is used, as the reference)
    std::string tag;
  };
  struct Record {
    std::vector<Segment> segs;
    std::string error;  // a line GenDesiredMatrix could not parse (reported when the record is used)
  };
  std::string mMlf;
  const char* mDir;
  const char* mExt;
  std::string mDirS, mExtS;
  std::unordered_map<std::string, int> mStates;
  std::vector<std::string> mTags;
  LabelIndex mIndex;  // MLF record patterns -> index into mRecords (labelindex.h)
  std::vector<Record> mRecords;
};

// The read-ahead pool.  Next() hands out utterances in script order; the pointer stays valid until
// the following Next() / Rewind().
class FeatureReader {
 public:
  FeatureReader(const std::string& scp, const FeatureConfig& cfg, std::shared_ptr<const MlfLabels> labels,
                int threads, int depth);
  ~FeatureReader();
  const Utterance* Next();  // nullptr at the end of the list; throws the record's error
  void Rewind();
  size_t Size() const { return mRecords.size(); }
  size_t Position() const { return mNext; }

 private:
  void Start();
  void Stop();
  void Worker();

  FeatureConfig mCfg;
  std::shared_ptr<const MlfLabels> mLabels;
  std::vector<FileRecord> mRecords;
  int mThreads, mDepth;
  int mTargetKind = kParmAnon, mDerivOrder = 0;  // latched from the first record
  std::string mLatchError;

  std::mutex mMu;
  std::condition_variable mCvWork, mCvDone;
  std::vector<std::thread> mPool;
  bool mStop = false;
  size_t mIssued = 0;  // next record index a worker takes
  size_t mNext = 0;    // next record index the consumer takes
  struct Slot {
    std::unique_ptr<Utterance> u;
    std::string error;
  };
  std::map<size_t, Slot> mDone;
  std::unique_ptr<Utterance> mCurrent;
  std::vector<std::unique_ptr<Utterance>> mFree;  // recycled utterance buffers
};

}  // namespace tnetio
