// htkio_sanitize.cpp -- host-only stress driver for the native reader (csrc/host/htkio.cpp) built with
// the compiler's sanitizers (tools/htkio_sanitize.sh: ThreadSanitizer for the read-ahead pool,
// AddressSanitizer + UndefinedBehaviorSanitizer for the decoders).  No device code is involved.
//
// usage: htkio_sanitize <dir> <scp> <mlf> <states> <start_ext> <end_ext>
// Reads the list with several pool shapes, rewinds mid-list, abandons a reader mid-list (destructor
// with workers still reading ahead), and checks every pass delivers the same frames in script order.
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "htkio.h"

static double checksum(const tnetio::Utterance& u) {
  double s = 0;
  for (size_t i = 0; i < u.feats.size(); i++) s += u.feats[i] * (double)((i % 7) + 1);
  for (size_t i = 0; i < u.labels.size(); i++) s += u.labels[i] * 1e-3;
  return s;
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s dir scp mlf states start_ext end_ext\n", argv[0]);
    return 2;
  }
  if (chdir(argv[1]) != 0) return 2;
  tnetio::FeatureConfig cfg;
  cfg.startExt = atoi(argv[5]);
  cfg.endExt = atoi(argv[6]);
  auto labels = std::make_shared<tnetio::MlfLabels>(argv[3], argv[4], nullptr, "lab");
  std::vector<double> ref;
  {
    tnetio::FeatureReader r(argv[2], cfg, labels, 1, 1);
    while (const tnetio::Utterance* u = r.Next()) ref.push_back(checksum(*u));
  }
  const int shapes[][2] = {{2, 1}, {4, 3}, {8, 16}, {16, 64}};
  for (auto& sh : shapes) {
    tnetio::FeatureReader r(argv[2], cfg, labels, sh[0], sh[1]);
    for (int pass = 0; pass < 2; pass++) {
      size_t k = 0;
      while (const tnetio::Utterance* u = r.Next()) {
        if (k >= ref.size() || checksum(*u) != ref[k]) {
          fprintf(stderr, "mismatch at record %zu (threads %d depth %d pass %d)\n", k, sh[0], sh[1], pass);
          return 1;
        }
        k++;
        if (pass == 0 && k == ref.size() / 2) break;  // rewind mid-list
      }
      r.Rewind();
    }
    // abandon mid-list: the destructor stops workers that are still reading ahead
    tnetio::FeatureReader a(argv[2], cfg, labels, sh[0], sh[1]);
    for (int i = 0; i < 3 && a.Next(); i++) {
    }
  }
  printf("htkio_sanitize ok: %zu records, %zu pool shapes\n", ref.size(), sizeof(shapes) / sizeof(shapes[0]));
  return 0;
}
