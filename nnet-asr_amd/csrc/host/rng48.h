// rng48.h -- explicit-state restatement of the drand48 family the reference draws its data order
// from: srand48(SEED) at TNetCu.cc:330-338, lrand48() % n in CuCache::GenerateRandom
// (cuCache.h:46-48) and CuRand seeding (curand.tcc:13-49).  glibc's published algorithm:
// X_{n+1} = (0x5DEECE66D X_n + 0xB) mod 2^48, srand48(s): X = (s << 16) | 0x330E,
// lrand48() = X >> 17.  Holding the state in an object (instead of libc's hidden global) keeps
// several trainers / ranks in one process independent and reproducible.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <vector>

namespace TNet {

class Rng48 {
 public:
  explicit Rng48(long seed = 0) { Seed(seed); }
  void Seed(long seed) { mX = ((((uint64_t)(uint32_t)seed) << 16) | 0x330Eu) & kMask; }
  /// raw 48-bit state (tests / checkpointing)
  uint64_t State() const { return mX; }
  void SetState(uint64_t x) { mX = x & kMask; }
  long Lrand48() {
    if (mLibc) return ::lrand48();
    mX = (0x5DEECE66Dull * mX + 0xBull) & kMask;
    return (long)(mX >> 17);
  }
  /// Draw from the C library's srand48/lrand48 stream instead (drop-in build: the reference
  /// drivers seed it with srand48(SEED), TNetCu.cc:330-338, and CuCache shuffles with lrand48)
  void UseLibc(bool on) { mLibc = on; }
  bool Libc() const { return mLibc; }
  /// libstdc++ std::random_shuffle(first, last, gen) with gen(k) = lrand48() % k
  /// (bits/stl_algo.h:4603-4620)
  void RandomShuffle(int* p, size_t n) {
    for (size_t i = 1; i < n; i++) {
      size_t j = (size_t)(Lrand48() % (long)(i + 1));
      if (i != j) {
        int t = p[i];
        p[i] = p[j];
        p[j] = t;
      }
    }
  }

 private:
  static constexpr uint64_t kMask = 0xFFFFFFFFFFFFull;
  uint64_t mX = 0;
  bool mLibc = false;
};

/// Process-wide stream, the counterpart of libc's srand48/lrand48 state.
Rng48& GlobalRng();
void SeedRandom(long seed);

}  // namespace TNet
