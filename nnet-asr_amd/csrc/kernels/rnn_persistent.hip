// rnn_persistent.hip -- one TRecurrentCu utterance in ONE launch (BASELINE config 5).
//
// The reference runs every frame as ~18 synchronous single-row cuBLAS / kernel calls
// (TRecurrentCu.cc:319-375 over cuRecurrent.cc:16-153 and cuBiasedLinearity.cc:11-64); the
// launch-per-op chain of gemv.hip still pays ~4 us per dependent launch, 9 a frame.  Here G
// co-resident workgroups keep the weights in LDS for the whole utterance and meet only at the
// frame's true data dependencies:
//   workgroup g owns recurrent columns J_g (jc of the H) and output columns C_g (cc of the N);
//   W[:, J_g] ([nIn + H] x jc) and Wo[:, C_g] (H x cc) live in LDS, written back at the end.
// Per frame t (7 exchanges at BPTT 4, each an all-to-all hand-off of 8-byte {tag, value} granules
// stored write-through and polled relaxed -- cdna_hip_programming.md Guideline 16, form R2):
//   1. y_t[J_g] = sigmoid(b + [x_t, y_{t-1}] W[:, J_g])                        -> AG1 (y_t, H)
//   2. gather y_t; z_c = bo_c + y_t Wo[:, c] for c in C_g; {max, sum exp} pair -> AG2 (2 per g)
//   3. the softmax normaliser from the G pairs; e_c = y_c - [c == label]; cross-entropy and the
//      frame's argmax key; P[k] = sum_c Wo[k, c] e_c (OLD Wo), then the Wo / bo SGD in LDS
//                                                                                -> RS (P, H per g)
//   4. d_0[J_g] = (sum_g P_g[J_g]) y_t (1 - y_t); for tau = 1..bptt: Q[i] = sum_{j in J_g}
//      W[nIn + i, j] d_{tau-1}[j] -> RS; d_tau[J_g] = (sum_g Q_g[J_g]) y_{t-tau} (1 - y_{t-tau})
//   5. W[:, J_g] += sum_tau (-lr h_tau) (x) d_tau - lr wc W ; b, cb   (rnn_update_kernel's order)
// Every hand-off is all-to-all, so a buffer is reused only after an exchange every workgroup has
// completed in between; the reduce-scatter buffers alternate.  Spins are bounded (2 s of
// s_memrealtime): a workgroup that times out sets *err and leaves; the others time out after it.
// Arithmetic is the single-frame chain's per element; only the GEMV summation order differs (dot
// products split over workgroups), inside the RNN tests' tolerances.
#include <float.h>

#include "kcommon.h"

namespace tnetk {

struct RnnPersistP {
  int nIn, H, N, T, bptt, G, jc, cc, R;  // R = history ring rows of y (bptt + 2)
  const float* X;
  long ldx;
  const int* labels;
  float* W;
  long ldw;
  float* b;
  float* cb;
  float* Wo;
  long ldwo;
  float* bo;
  float* Woc;  // output-layer momentum buffers (nullable)
  long ldwoc;
  float* boc;
  float lr, mmt, wc;        // CuRecurrent::Update
  float oscale, ommt, ol2;  // CuBiasedLinearity::UpdateConstants(1)
  float* y;                 // [H] y_{-1} in, y_{T-1} out (the recurrent layer's output)
  double* stats;
  unsigned long long* argkey;  // [T], zeroed by the caller
  unsigned long long* xbuf;    // exchange granules: AG1 [H], AG2 [2 G], RS [2][G H]
  unsigned epoch0;
  int train;
  int* err;
  long long* stamps;  // diagnostics (tnet_rnn_utterance_stamps): workgroup 0's s_memrealtime per phase
};

typedef unsigned long long u64;
constexpr long kSpinTicks = 200000000;  // 2 s of the 100 MHz s_memrealtime

__device__ __forceinline__ void put(u64* g, unsigned tag, float v) {
  __hip_atomic_store(g, ((u64)tag << 32) | (u64)__float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 get(const u64* g) {
  return __hip_atomic_load(const_cast<u64*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every thread loads its n granules (addresses from idx(k)) until all carry `tag`; values to out[k].
// Returns false on timeout (err set).  All threads of the workgroup call it.
template <int MAXN, typename F>
__device__ __forceinline__ bool gather(const u64* buf, int n, F idx, unsigned tag, float (&out)[MAXN],
                                       int* err, long t_start) {
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < MAXN; ++k)
      if (k < n) {
        const u64 v = get(buf + idx(k));
        out[k] = __uint_as_float((unsigned)(v & 0xffffffffull));
        ok = ok && (unsigned)(v >> 32) == tag;
      }
    if (__syncthreads_and(ok)) return true;
    if ((long)__builtin_amdgcn_s_memrealtime() - t_start > kSpinTicks) {
      if (threadIdx.x == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ __launch_bounds__(256) void rnn_utterance_kernel(const RnnPersistP p) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = blockIdx.x, G = p.G, H = p.H, N = p.N, nIn = p.nIn, D = nIn + H, jc = p.jc, cc = p.cc, R = p.R;
  const int j0 = g * jc, c0 = g * cc;
  const int jn = max(0, min(jc, H - j0)), cn = max(0, min(cc, N - c0));  // this group's live columns
  // LDS carve: Ws [jc][D], Wos [cc][H], yr [R][H], xr [R][nIn], zs [cc], es [cc], ds [(bptt+1)][jc],
  // red [G][jc]
  float* Ws = sm;
  float* Wos = Ws + (long)jc * D;
  float* yr = Wos + (long)cc * H;
  float* xr = yr + (long)R * H;
  float* zs = xr + (long)R * nIn;
  float* es = zs + cc;
  float* ds = es + cc;
  float* red = ds + (p.bptt + 1) * jc;
  __shared__ float s_norm[2], s_red[4];
  __shared__ double s_redd[4];
  __shared__ ArgMax s_arg[4];

  u64* AG1 = p.xbuf;
  u64* AG2 = AG1 + H;
  u64* RS0 = AG2 + 2 * G;
  const long rs_stride = (long)G * H;

  for (long i = tid; i < (long)jc * D; i += 256) {
    const int c = (int)(i / D), d = (int)(i % D);
    Ws[i] = c < jn ? p.W[(long)d * p.ldw + j0 + c] : 0.f;
  }
  for (long i = tid; i < (long)cc * H; i += 256) {
    const int c = (int)(i / H), k = (int)(i % H);
    Wos[i] = c < cn ? p.Wo[(long)k * p.ldwo + c0 + c] : 0.f;
  }
  for (int i = tid; i < R * H; i += 256) yr[i] = 0.f;
  __syncthreads();
  for (int k = tid; k < H; k += 256) yr[(long)((R - 1) % R) * H + k] = p.y[k];  // y_{-1} in ring row R-1
  __syncthreads();

  auto yrow = [&](int f) -> const float* { return yr + (long)(((f % R) + R) % R) * H; };  // y_f, f >= -1
  auto xrow = [&](int f) -> const float* { return xr + (long)(f % R) * nIn; };             // x_f, f >= 0
  int rs_count = 0;
  bool alive = true;
  auto stamp = [&](int t, int k) {
    if (p.stamps && g == 0 && tid == 0) p.stamps[(long)t * 8 + k] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  for (int t = 0; t < p.T && alive; ++t) {
    const long t_start = (long)__builtin_amdgcn_s_memrealtime();
    stamp(t, 0);
    const unsigned tag0 = p.epoch0 + (unsigned)t * 16u + 1u;  // 16 tags a frame: AG1, AG2, RS 0..bptt (<= 8)
    // x_t into the LDS ring (the frame's dot products and the update read the last bptt+1 rows there)
    {
      float* xw = xr + (long)(t % R) * nIn;
      for (int d = tid; d < nIn; d += 256) xw[d] = p.X[(long)t * p.ldx + d];
    }
    __syncthreads();
    const float* xt = xrow(t);
    const float* yprev = yrow(t - 1);
    // ---- 1. own recurrent outputs y_t[J_g]
    for (int c = wv; c < jn; c += 4) {
      const float* w = Ws + (long)c * D;
      float a = 0.f;
      for (int d = lane; d < nIn; d += 64) a += w[d] * xt[d];
      for (int d = lane; d < H; d += 64) a += w[nIn + d] * yprev[d];
      a = wave_sum(a);
      if (lane == 0) put(AG1 + j0 + c, tag0, sigmoidf_ref(p.b[j0 + c] + a));
    }
    // ---- 2. gather y_t; output logits of C_g and their {max, sum exp}
    stamp(t, 1);
    {
      float v[4];
      const int nk = (H + 255) / 256;
      if (!gather<4>(AG1, nk, [&](int k) { return min(tid + 256 * k, H - 1); }, tag0, v, p.err, t_start)) {
        alive = false;
        break;
      }
      float* yt = yr + (long)(t % R) * H;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (k < nk && tid + 256 * k < H) yt[tid + 256 * k] = v[k];
    }
    __syncthreads();
    stamp(t, 2);
    const float* yt = yr + (long)(t % R) * H;
    for (int c = wv; c < cn; c += 4) {
      const float* w = Wos + (long)c * H;
      float a = 0.f;
      for (int k = lane; k < H; k += 64) a += w[k] * yt[k];
      a = wave_sum(a);
      if (lane == 0) zs[c] = p.bo[c0 + c] + a;
    }
    __syncthreads();
    if (wv == 0) {
      float m = -1e30f;
      for (int c = lane; c < cn; c += 64) m = fmaxf(m, zs[c]);
      m = wave_max(m);
      float s = 0.f;
      for (int c = lane; c < cn; c += 64) s += fast_exp(zs[c] - m);
      s = (float)wave_sum_d((double)s);
      if (lane == 0) {
        put(AG2 + 2 * g, tag0 + 1, m);
        put(AG2 + 2 * g + 1, tag0 + 1, s);
      }
    }
    // ---- 3. softmax normaliser, error, statistics, output-layer backprop partials + SGD
    stamp(t, 3);
    {
      float v[2];
      if (!gather<2>(AG2, tid < G ? 2 : 0, [&](int k) { return 2 * tid + k; }, tag0 + 1, v, p.err, t_start)) {
        alive = false;
        break;
      }
      // the normaliser: M = max m_q, S = sum s_q exp(m_q - M) over the G pairs (thread q holds pair q)
      const float mg = tid < G ? v[0] : -1e30f;
      float m = wave_max(mg);
      if (lane == 0) s_red[wv] = m;
      __syncthreads();
      const float Mx = fmaxf(fmaxf(s_red[0], s_red[1]), fmaxf(s_red[2], s_red[3]));
      const double sw = wave_sum_d(tid < G ? (double)v[1] * (double)fast_exp(mg - Mx) : 0.0);
      if (lane == 0) s_redd[wv] = sw;
      __syncthreads();
      if (tid == 0) {
        s_norm[0] = Mx;
        s_norm[1] = 1.f / (float)(((s_redd[0] + s_redd[1]) + s_redd[2]) + s_redd[3]);
      }
    }
    __syncthreads();
    const float M = s_norm[0], rsum = s_norm[1];
    const int lab = p.labels[t];
    const int tl = lab < N ? lab : -1;
    {
      ArgMax ay{-1e20f, 0x7fffffff};
      for (int c = tid; c < cn; c += 256) {
        const float yc = fast_exp(zs[c] - M) * rsum;
        es[c] = yc - (c0 + c == tl ? 1.f : 0.f);
        if (yc > ay.v) {
          ay.v = yc;
          ay.i = c0 + c;
        }
        if (c0 + c == tl && p.stats) atomicAdd(p.stats, -(double)logf(fmaxf(yc, FLT_MIN)));
      }
      ay = wave_argmax(ay);
      if (lane == 0) s_arg[wv] = ay;
      __syncthreads();
      if (tid == 0 && cn > 0) {
        ArgMax a = s_arg[0];
#pragma unroll
        for (int q = 1; q < 4; ++q) a = argmax_merge(a, s_arg[q]);
        atomicMax(p.argkey + t, ((u64)__float_as_uint(fmaxf(a.v, 0.f)) << 32) | (u64)(0xffffffffu - (unsigned)a.i));
      }
    }
    stamp(t, 4);
    if (!p.train) continue;
    u64* RS = RS0 + (long)(rs_count & 1) * rs_stride;
    for (int k = tid; k < H; k += 256) {
      const float xk = yt[k];
      float acc = 0.f;
      for (int c = 0; c < cn; ++c) {
        float* wp = Wos + (long)c * H + k;
        const float w = *wp, ec = es[c];
        acc += w * ec;
        float cv = xk * ec;
        if (p.Woc) {
          float* qp = p.Woc + (long)k * p.ldwoc + c0 + c;
          cv = cv + p.ommt * *qp;
          *qp = cv;
        }
        float wn = w + p.oscale * cv;
        *wp = wn + p.ol2 * wn;
      }
      put(RS + (long)g * H + k, tag0 + 2, acc);
    }
    for (int c = tid; c < cn; c += 256) {
      float gb = es[c];
      if (p.boc) {
        gb = gb + p.ommt * p.boc[c0 + c];
        p.boc[c0 + c] = gb;
      }
      p.bo[c0 + c] = p.bo[c0 + c] + p.oscale * gb;
    }
    // ---- 4. d_0 and the BPTT chain, each step one reduce-scatter of H partials
    stamp(t, 5);
    for (int tau = 0; tau <= p.bptt; ++tau) {
      const u64* RSr = RS0 + (long)(rs_count & 1) * rs_stride;
      float v[8];
      const int nv = jn > 0 ? (G * jc + 255) / 256 : 0;  // granules per thread: (producer q, own column c)
      if (!gather<8>(RSr, nv, [&](int k) {
            const int i = min(tid + 256 * k, G * jc - 1);
            return (long)(i / jc) * H + j0 + min(i % jc, max(jn - 1, 0));
          }, tag0 + 2 + (unsigned)tau, v, p.err, t_start)) {
        alive = false;
        break;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < nv && tid + 256 * k < G * jc) red[tid + 256 * k] = v[k];
      __syncthreads();
      ++rs_count;
      const float* yh = tau == 0 ? yt : (t - tau >= 0 ? yrow(t - tau) : nullptr);
      if (tid < jn) {
        float s = 0.f;
        for (int q = 0; q < G; ++q) s += red[q * jc + tid];  // producers in order
        const float yv = yh ? yh[j0 + tid] : 0.f;
        ds[tau * jc + tid] = s * (yv * (1.f - yv));
      }
      __syncthreads();
      if (tau == p.bptt) break;
      u64* RSw = RS0 + (long)(rs_count & 1) * rs_stride;
      for (int i = tid; i < H; i += 256) {
        float a = 0.f;
        for (int c = 0; c < jn; ++c) a += Ws[(long)c * D + nIn + i] * ds[tau * jc + c];
        put(RSw + (long)g * H + i, tag0 + 3 + (unsigned)tau, a);
      }
    }
    if (!alive) break;
    stamp(t, 6);
    // ---- 5. recurrent weight + bias update (rnn_update_kernel's per-element order)
    for (int d = tid; d < D; d += 256) {
      float hv[9];  // history rows tau = [x_f, y_{f-1}] at column d, f = t - tau (zero before the utterance)
#pragma unroll
      for (int tau = 0; tau < 9; ++tau) {
        const int f = t - tau;
        hv[tau] = 0.f;
        if (tau <= p.bptt && f >= 0) hv[tau] = d < nIn ? xrow(f)[d] : yrow(f - 1)[d - nIn];
      }
      for (int c = 0; c < jn; ++c) {
        float acc = 0.f;
#pragma unroll
        for (int tau = 0; tau < 9; ++tau)
          if (tau <= p.bptt) acc += (-p.lr * hv[tau]) * ds[tau * jc + c];
        const float w = Ws[(long)c * D + d];
        const float corr = (-p.lr * p.wc) * w + acc;
        Ws[(long)c * D + d] = corr + w;
      }
    }
    if (tid < jn) {
      float gb = -p.lr * ds[tid] + p.mmt * p.cb[j0 + tid];
      for (int tau = 1; tau <= p.bptt; ++tau) gb = -p.lr * ds[tau * jc + tid] + gb;
      p.cb[j0 + tid] = gb;
      p.b[j0 + tid] = gb + p.b[j0 + tid];
    }
    __syncthreads();
    stamp(t, 7);
  }
  // ---- write back (the training launch's W / Wo slices; y_{T-1} by group 0)
  if (p.train) {
    for (long i = tid; i < (long)jn * D; i += 256) {
      const int c = (int)(i / D), d = (int)(i % D);
      p.W[(long)d * p.ldw + j0 + c] = Ws[i];
    }
    for (long i = tid; i < (long)cn * H; i += 256) {
      const int c = (int)(i / H), k = (int)(i % H);
      p.Wo[(long)k * p.ldwo + c0 + c] = Wos[i];
    }
  }
  if (g == 0 && p.T > 0) {
    const float* yl = yr + (long)((p.T - 1) % R) * H;
    for (int k = tid; k < H; k += 256) p.y[k] = yl[k];
  }
}

}  // namespace tnetk

using namespace tnetk;

static long long* g_rnn_stamps = nullptr;
extern "C" int tnet_rnn_utterance_stamps(long long* buf) {
  g_rnn_stamps = buf;
  return TNET_OK;
}

extern "C" long tnet_rnn_utterance_workspace(int H, int N, int G) {
  (void)N;
  return (long)(H + 2 * G + 2L * G * H) * 8;
}

extern "C" int tnet_rnn_utterance(const float* X, int T, int nIn, int ldx, const int* labels, float* W, int ldw,
                                  float* b, float* corr_b, int H, float* Wo, int ldwo, float* bo, float* corr_Wo,
                                  int ldwoc, float* corr_bo, int N, int bptt, float lr, float mmt, float wc,
                                  float oscale, float ommt, float ol2, float* y, double* stats,
                                  unsigned long long* argkey, void* workspace, unsigned epoch0, int train,
                                  int* err, void* stream) {
  if (T < 0 || nIn <= 0 || H <= 0 || N <= 0 || bptt < 0 || bptt > 8 || !X || !labels || !W || !b || !corr_b ||
      !Wo || !bo || !y || !argkey || !workspace || !err || ldx < nIn || ldw < H || ldwo < N ||
      (ommt != 0.f && (!corr_Wo || !corr_bo || ldwoc < N)))
    return TNET_ERR_ARG;
  if (!T) return TNET_OK;
  // workgroups: the fewest (cheapest hand-offs) whose weight slices fit the LDS
  const int D = nIn + H, R = bptt + 2;
  int G = 0, jc = 0, cc = 0;
  size_t lds = 0;
  for (int g = 16; g <= 256; g *= 2) {
    jc = cdiv(H, g);
    cc = cdiv(N, g);
    lds = sizeof(float) * ((size_t)jc * D + (size_t)cc * H + (size_t)R * (H + nIn) + 2 * cc + (bptt + 1) * jc +
                           (size_t)g * jc);
    if (lds <= 150 * 1024) {
      G = g;
      break;
    }
  }
  if (!G || (long)G * jc > 256 * 8) return TNET_ERR_UNSUPPORTED;
  RnnPersistP p;
  p.nIn = nIn; p.H = H; p.N = N; p.T = T; p.bptt = bptt; p.G = G; p.jc = jc; p.cc = cc; p.R = R;
  p.X = X; p.ldx = ldx; p.labels = labels;
  p.W = W; p.ldw = ldw; p.b = b; p.cb = corr_b;
  p.Wo = Wo; p.ldwo = ldwo; p.bo = bo;
  p.Woc = ommt != 0.f ? corr_Wo : nullptr; p.ldwoc = ldwoc; p.boc = ommt != 0.f ? corr_bo : nullptr;
  p.lr = lr; p.mmt = mmt; p.wc = wc; p.oscale = oscale; p.ommt = ommt; p.ol2 = ol2;
  p.y = y; p.stats = stats; p.argkey = argkey; p.xbuf = (unsigned long long*)workspace; p.epoch0 = epoch0;
  p.train = train; p.err = err; p.stamps = g_rnn_stamps;
  hipStream_t st = (hipStream_t)stream;
  if (hipFuncSetAttribute((const void*)rnn_utterance_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return TNET_ERR_RUNTIME;
  void* args[] = {&p};
  // cooperative: the launch fails instead of leaving a workgroup un-resident (every frame waits on all)
  if (hipLaunchCooperativeKernel((const void*)rnn_utterance_kernel, dim3(G), dim3(256), args, (unsigned)lds, st) !=
      hipSuccess)
    return TNET_ERR_LAUNCH;
  return TNET_OK;
}
