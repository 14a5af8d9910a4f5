// xcd_handoff_probe.hip -- the floor of one all-to-all hand-off of the persistent RNN kernel (rnn_persistent.hip,
// AG1: every workgroup publishes its jc = H / G recurrent outputs as 8-byte {tag, value} granules, then every
// workgroup polls all H granules until they carry the frame's tag) for different placements of the G workgroups
// (is an XCD-local chain worth building?).
//
// 256 workgroups are launched (one per CU); only the `active` ones take part, the others return at once.
//   place 0 "one-xcd":  active = blockIdx % 8 == 0 (G = 32; workgroup i is dispatched to XCD i % 8, so these 32
//                       sit on one XCD -- placement is used for SPEED only in forms 0 / 1)
//   place 1 "spread":   active = blockIdx < G (G / 8 a XCD)
// Forms (how a granule travels):
//   0: relaxed agent-scope atomic store / load (rnn_persistent.hip's put / get: sc1, through memory-side MALL)
//   1: the same granules, then a vmcnt drain and one relaxed agent ticket per workgroup; consumers poll the one
//      counter (thread 0), then read every granule once (Guideline 16's counter form)
//   2: plain stores / loads with L1 bypass only (sc0): coherent ONLY if every workgroup shares one L2 -- the
//      placement-dependent form cdna_hip_programming.md rejects as a product protocol (its §5 item 2, Pitfall 1);
//      measured here with place 0 only, to price what the rule gives up.  A stale read shows as a timeout.
// Every spin is bounded (0.5 s of the 100 MHz s_memrealtime): a timeout sets err and the workgroup leaves.
// Output: ticks per round (10 ns each) from workgroup 0's s_memrealtime, one line per (form, place, G).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/xcd_handoff_probe tools/xcd_handoff_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned long long u64;
constexpr long kSpin = 50000000;  // 0.5 s
constexpr int kH = 512;           // recurrent width (config 5)
constexpr int kRounds = 2000;

struct P {
  u64* buf;       // [2][kH] granules (rounds alternate halves)
  unsigned* cnt;  // [kRounds] tickets (form 1)
  int form, place, G;
  int* err;
  long long* t;   // [2] workgroup 0's start / end
};

__device__ __forceinline__ bool active_id(const P& p, int b, int* g) {
  if (p.place == 0) {
    if (b % 8) return false;
    *g = b / 8;
  } else {
    if (b >= p.G) return false;
    *g = b;
  }
  return *g < p.G;
}

__global__ __launch_bounds__(256) void probe(P p) {
  int g;
  if (!active_id(p, (int)blockIdx.x, &g)) return;
  const int tid = threadIdx.x, jc = kH / p.G;
  __shared__ int s_ok;
  const long t0 = (long)__builtin_amdgcn_s_memrealtime();
  if (g == 0 && tid == 0) p.t[0] = t0;
  for (int r = 0; r < kRounds; ++r) {
    const unsigned tag = (unsigned)r + 1u;
    u64* half = p.buf + (long)(r & 1) * kH;
    // publish this workgroup's jc granules
    if (tid < jc) {
      const u64 v = ((u64)tag << 32) | (u64)__float_as_uint((float)(g * jc + tid));
      u64* dst = half + g * jc + tid;
      if (p.form == 0 || p.form == 1)
        __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else  // plain 8-B store (L1 is write-through: it lands in this XCD's L2)
        __builtin_amdgcn_raw_buffer_store_b64(
            (__attribute__((ext_vector_type(2))) unsigned){(unsigned)v, (unsigned)(v >> 32)},
            __builtin_amdgcn_make_buffer_rsrc((void*)half, (short)0, 0x7FFFFFF0, 0x00020000), (g * jc + tid) * 8, 0, 0);
    }
    if (p.form == 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(p.cnt + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // gather all kH granules (2 a thread)
    for (;;) {
      bool ok = true;
      if (p.form == 1) {
        if (tid == 0) {
          unsigned c;
          do {
            c = __hip_atomic_load(p.cnt + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (c >= (unsigned)p.G) break;
            if ((long)__builtin_amdgcn_s_memrealtime() - t0 > kSpin) break;
          } while (true);
          s_ok = c >= (unsigned)p.G;
        }
        __syncthreads();
        ok = s_ok;
      }
      if (ok) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)half, (short)0, 0x7FFFFFF0, 0x00020000);
        if (p.form == 2) asm volatile("buffer_inv sc0" ::: "memory");  // drop this CU's L1 lines
        for (int k = tid; k < kH; k += 256) {
          u64 v;
          if (p.form == 2) {
            const auto w = __builtin_amdgcn_raw_buffer_load_b64(rs, k * 8, 0, 0);  // plain: L1 was invalidated
            v = ((u64)w[1] << 32) | (u64)w[0];
          } else {
            v = __hip_atomic_load(half + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          ok = ok && (unsigned)(v >> 32) == tag;
        }
      }
      if (__syncthreads_and(ok)) break;
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > kSpin) {
        if (tid == 0) __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
    }
  }
  if (g == 0 && tid == 0) p.t[1] = (long)__builtin_amdgcn_s_memrealtime();
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

int main() {
  u64* buf;
  unsigned* cnt;
  int* err;
  long long* t;
  CK(hipMalloc(&buf, 2 * kH * sizeof(u64)));
  CK(hipMalloc(&cnt, kRounds * sizeof(unsigned)));
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMalloc(&t, 2 * sizeof(long long)));
  struct Case {
    int form, place, G;
  };
  const std::vector<Case> cases = {{0, 0, 32}, {0, 1, 32}, {0, 1, 128}, {1, 0, 32}, {1, 1, 32}, {1, 1, 128}, {2, 0, 32}};
  const char* fname[] = {"granule-atomic(sc1)", "sc1-data+ticket", "plain-L2-only(placement-dependent)"};
  const char* pname[] = {"one-xcd", "spread"};
  for (const Case& c : cases) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(buf, 0, 2 * kH * sizeof(u64)));
      CK(hipMemset(cnt, 0, kRounds * sizeof(unsigned)));
      CK(hipMemset(err, 0, sizeof(int)));
      CK(hipMemset(t, 0, 2 * sizeof(long long)));
      P p{buf, cnt, c.form, c.place, c.G, err, t};
      probe<<<256, 256>>>(p);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      int e = 0;
      long long tt[2];
      CK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
      CK(hipMemcpy(tt, t, sizeof tt, hipMemcpyDeviceToHost));
      std::printf("{\"form\": \"%s\", \"place\": \"%s\", \"G\": %d, \"rep\": %d, \"timeout\": %d, \"us_per_round\": %.3f}\n",
                  fname[c.form], pname[c.place], c.G, rep, e, e ? -1.0 : (tt[1] - tt[0]) * 0.01 / kRounds);
      std::fflush(stdout);
    }
  }
  return 0;
}
