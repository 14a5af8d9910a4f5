#!/bin/bash
# Host-only sanitizer runs of the native reader (csrc/host/htkio.cpp) on examples/01's files:
# ThreadSanitizer (the read-ahead pool) and AddressSanitizer + UndefinedBehaviorSanitizer (decoders).
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
B=$(mktemp -d)
SRC="$R/tools/htkio_sanitize.cpp $R/nnet-asr_amd/csrc/host/htkio.cpp $R/nnet-asr_amd/csrc/host/labelindex.cpp"
INC="-I$R/nnet-asr_amd/csrc/host"
EX="$R/tests/golden/ex01"
g++ -std=c++17 -O1 -g -fsanitize=thread $INC $SRC -o "$B/tsan" -pthread
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=undefined $INC $SRC -o "$B/asan" -pthread
for ext in "0 0" "25 25"; do
  TSAN_OPTIONS="halt_on_error=1" "$B/tsan" "$EX" test.scp test_3s.mlf mono_state_phn_set_135_phn $ext
  ASAN_OPTIONS="detect_leaks=1" "$B/asan" "$EX" test.scp test_3s.mlf mono_state_phn_set_135_phn $ext
done
rm -rf "$B"
