/*
 * tnet_oracle.c -- CPU restatement of the reference TNet frame-batched SGD path.
 *
 * TEST INFRASTRUCTURE ONLY.  Imported (via ctypes, oracle/oracle.py) by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg -- always as the checker, never as
 * the thing measured or shipped.  The product (nnet-asr_amd/) never links or loads it.
 *
 * Parity pinning: the CPU-semantics path (cpu_semantics=1) is checked bit-for-bit-ish
 * (float tolerance) against golden vectors produced by the reference TNetLib itself
 * (tests/golden/steps_*.npz, shuffle.npz; generator tests/golden/make_golden.py).  The
 * GPU-semantics path (momentum, GRADDIVFRM, double column sums, FLT_MIN-clamped Xent) is
 * restated from the CuTNetLib/CUDA sources, which cannot run here; it reduces to the pinned
 * CPU path at momentum=0, GRADDIVFRM=F (run_test.GPU.sh:50) and is otherwise "parity unpinned"
 * beyond that equivalence.
 *
 * Accumulation: GEMMs and reductions accumulate in double (a tighter checker than the
 * reference's float BLAS); element-wise maps follow the reference formulas.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------------------------
 * drand48 family (glibc published algorithm): X_{n+1} = (a X_n + c) mod 2^48,
 * a = 0x5DEECE66D, c = 0xB; srand48(s): X = (s << 16) | 0x330E; lrand48 = X >> 17.
 * The reference seeds with srand48(SEED) (src/TNetCu.cc:330-338, src/TNetLib/Cache.cc:40-50)
 * and draws lrand48() % n in the cache shuffle (src/CuTNetLib/cuCache.h:46-48).
 * ------------------------------------------------------------------------------------- */
typedef struct { uint64_t x; } orc_rng48;

void orc_srand48(orc_rng48* r, long seed) {
  r->x = (((uint64_t)(uint32_t)seed) << 16 | 0x330Eu) & 0xFFFFFFFFFFFFull;
}

long orc_lrand48(orc_rng48* r) {
  r->x = (0x5DEECE66Dull * r->x + 0xBull) & 0xFFFFFFFFFFFFull;
  return (long)(r->x >> 17);
}

/* libstdc++ std::random_shuffle(first, last, gen) (bits/stl_algo.h:4603-4620) with
 * gen(k) = lrand48() % k, as called by CuCache::Randomize (src/CuTNetLib/cuCache.cc:124-152). */
void orc_random_shuffle(orc_rng48* r, int* p, int n) {
  for (int i = 1; i < n; i++) {
    int j = (int)(orc_lrand48(r) % (long)(i + 1));
    if (i != j) { int t = p[i]; p[i] = p[j]; p[j] = t; }
  }
}

/* Run the whole cache/bunch schedule of one epoch for utterance lengths lens[0..nutt):
 * CuCache::AddData/Randomize/GetBunch (cuCache.cc:41-200) + the TNetCu fill loop
 * (TNetCu.cc:376-441).  Emits, for every trained bunch, `bunch` global frame indices
 * (utterance frames concatenated in scp order).  Returns number of bunches written. */
long orc_epoch_schedule_x(const int* lens, int nutt, int cachesize, int bunch, uint64_t x0, int randomize,
                          int* out, long out_cap_bunches, uint64_t* x_end);

long orc_epoch_schedule(const int* lens, int nutt, int cachesize, int bunch, long seed, int randomize,
                        int* out, long out_cap_bunches) {
  orc_rng48 r; orc_srand48(&r, seed);
  return orc_epoch_schedule_x(lens, nutt, cachesize, bunch, r.x, randomize, out, out_cap_bunches, NULL);
}

/* Same schedule with the lrand48 stream starting at raw state x0 (TRbmCu draws the CuRand seeds
 * from the stream before the first shuffle, TRbmCu.cc:260-264); x_end receives the final state. */
long orc_epoch_schedule_x(const int* lens, int nutt, int cachesize, int bunch, uint64_t x0, int randomize,
                          int* out, long out_cap_bunches, uint64_t* x_end) {
  orc_rng48 r; r.x = x0;
  int* cache = (int*)malloc(sizeof(int) * (size_t)cachesize);
  int* perm = (int*)malloc(sizeof(int) * (size_t)cachesize);
  int* leftover = NULL; int nleft = 0;
  long nb = 0, fr0 = 0; int u = 0;
  while (u < nutt) {
    /* fill: state EMPTY -> prefill leftover (truncated to cachesize) */
    int intake = 0;
    if (nleft > 0) {
      int l = nleft < cachesize ? nleft : cachesize;
      /* a leftover that fills the whole cache leaves cache_space == 0 for the next utterance:
       * the reference aborts (cuCache.cc:97 / Cache.cc:117 assert(cache_space > 0)) */
      if (l == cachesize && u < nutt) { free(leftover); free(cache); free(perm); return -1; }
      memcpy(cache, leftover, sizeof(int) * (size_t)l);
      intake = l;
      free(leftover); leftover = NULL; nleft = 0;
    }
    while (intake < cachesize && u < nutt) {
      int space = cachesize - intake, len = lens[u];
      int fill = space < len ? space : len;
      for (int k = 0; k < fill; k++) cache[intake + k] = (int)(fr0 + k);
      if (len > fill) {
        nleft = len - fill;
        leftover = (int*)malloc(sizeof(int) * (size_t)nleft);
        for (int k = 0; k < nleft; k++) leftover[k] = (int)(fr0 + fill + k);
      }
      intake += fill; fr0 += len; u++;
    }
    for (int k = 0; k < intake; k++) perm[k] = k;
    if (randomize) orc_random_shuffle(&r, perm, intake);
    /* GetBunch until fewer than `bunch` rows remain (tail discarded) */
    for (int pos = 0; pos + bunch <= intake; pos += bunch) {
      if (nb < out_cap_bunches)
        for (int k = 0; k < bunch; k++) out[nb * bunch + k] = cache[perm[pos + k]];
      nb++;
    }
  }
  free(leftover); free(cache); free(perm);
  if (x_end) *x_end = r.x;
  return nb;
}

/* ---------------------------------------------------------------------------------------
 * Dense linear algebra (row-major).  C = alpha*op(A)*op(B) + beta*C, double accumulation.
 * Reference: CuMatrix::Gemm (src/CuBaseLib/cumatrix.tcc:336-370), Matrix::BlasGemm
 * (src/KaldiLib/Matrix.cc:161-199).
 * ------------------------------------------------------------------------------------- */
void orc_sgemm(char ta, char tb, int M, int N, int K, float alpha, const float* A, int lda,
               const float* B, int ldb, float beta, float* C, int ldc) {
  int tA = (ta == 'T' || ta == 't'), tB = (tb == 'T' || tb == 't');
  /* pack op(A) as [M x K] and op(B)^T as [N x K] (both K-contiguous), then double dots */
  float* Ap = (float*)malloc(sizeof(float) * (size_t)M * K);
  float* Bp = (float*)malloc(sizeof(float) * (size_t)N * K);
  for (int i = 0; i < M; i++)
    for (int k = 0; k < K; k++) Ap[(size_t)i * K + k] = tA ? A[(size_t)k * lda + i] : A[(size_t)i * lda + k];
  for (int j = 0; j < N; j++)
    for (int k = 0; k < K; k++) Bp[(size_t)j * K + k] = tB ? B[(size_t)j * ldb + k] : B[(size_t)k * ldb + j];
#pragma omp parallel for schedule(dynamic, 4)
  for (int i = 0; i < M; i++) {
    const float* a = Ap + (size_t)i * K;
    for (int j = 0; j < N; j++) {
      const float* bb = Bp + (size_t)j * K;
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      int k = 0;
      for (; k + 4 <= K; k += 4) {
        s0 += (double)a[k] * bb[k];
        s1 += (double)a[k + 1] * bb[k + 1];
        s2 += (double)a[k + 2] * bb[k + 2];
        s3 += (double)a[k + 3] * bb[k + 3];
      }
      for (; k < K; k++) s0 += (double)a[k] * bb[k];
      double acc = (s0 + s1) + (s2 + s3);
      float* c = C + (size_t)i * ldc + j;
      *c = (float)(alpha * acc + (beta == 0.0f ? 0.0 : (double)beta * *c));
    }
  }
  free(Ap); free(Bp);
}

/* y = b + X W  (CuBiasedLinearity::PropagateFnc, cuBiasedLinearity.cc:11-16) */
void orc_affine(const float* X, int rows, int n_in, const float* W, const float* b, int n_out, float* Y) {
  orc_sgemm('N', 'N', rows, n_out, n_in, 1.0f, X, n_in, W, n_out, 0.0f, Y, n_out);
  for (int r = 0; r < rows; r++)
    for (int c = 0; c < n_out; c++) Y[(size_t)r * n_out + c] += b[c];
}

/* _sigmoid (cukernels.cu:192-206): 1.0/(1.0+exp(-x)) with double constants */
void orc_sigmoid(float* y, const float* x, long n) {
  for (long i = 0; i < n; i++) y[i] = (float)(1.0 / (1.0 + exp(-(double)x[i])));
}

/* _diff_sigmoid (cukernels.cu:209-217): e_out = y (1 - y) e */
void orc_diff_sigmoid(float* eout, const float* e, const float* y, long n) {
  for (long i = 0; i < n; i++) eout[i] = (float)((double)y[i] * (1.0 - (double)y[i]) * (double)e[i]);
}

/* _softmax (cukernels.cu:220-242): double max / sum, y = exp(x - max) / sum */
void orc_softmax(float* y, const float* x, int rows, int cols) {
  for (int r = 0; r < rows; r++) {
    const float* xr = x + (size_t)r * cols;
    float* yr = y + (size_t)r * cols;
    double mx = -1e20, sum = 0.0;
    for (int c = 0; c < cols; c++) if (mx < xr[c]) mx = xr[c];
    for (int c = 0; c < cols; c++) { double e = exp((double)xr[c] - mx); yr[c] = (float)e; sum += yr[c]; }
    for (int c = 0; c < cols; c++) yr[c] = (float)((double)yr[c] / sum);
  }
}

/* v = alpha * sum_rows(M) + beta * v, double accumulation (_add_col_sum, cukernels.cu:147-164) */
void orc_add_col_sum(float alpha, const float* M, int rows, int cols, float beta, float* v) {
  for (int c = 0; c < cols; c++) {
    double s = 0.0;
    for (int r = 0; r < rows; r++) s += M[(size_t)r * cols + c];
    v[c] = (float)(alpha * s + (double)beta * v[c]);
  }
}

/* Cross-entropy objective with one-hot class-id targets (lab < 0: unlabeled, all-zero row).
 *   err = y - d                                   (cuObjectiveFunction.cc:62-63)
 *   correct += argmax(y) == argmax(d), first max   (_check_class, cukernels.cu:396-419;
 *                                                   FindMaxId, src/TNetLib/ObjFun.cc:64-74)
 *   xent += -sum_c d log(max(y, FLT_MIN))          (cuObjectiveFunction.cc:72-80, _log_elem)
 */
void orc_xent_eval(const float* y, const int* lab, int rows, int cols, float* err, double* xent,
                   long* correct) {
  for (int r = 0; r < rows; r++) {
    const float* yr = y + (size_t)r * cols;
    int t = lab[r];
    int am = -1; float mv = -1e20f;
    for (int c = 0; c < cols; c++) if (yr[c] > mv) { mv = yr[c]; am = c; }
    int des = t >= 0 ? t : 0;  /* all-zero target row: first max of zeros is column 0 */
    if (am == des) (*correct)++;
    if (t >= 0) {
      float p = yr[t] < FLT_MIN ? FLT_MIN : yr[t];
      *xent -= log((double)p);
    }
    if (err)
      for (int c = 0; c < cols; c++) err[(size_t)r * cols + c] = yr[c] - (c == t ? 1.0f : 0.0f);
  }
}

/* ---------------------------------------------------------------------------------------
 * One SGD step of a <biasedlinearity>/<sigmoid>... /<biasedlinearity>/<softmax> MLP with
 * cross-entropy.  dims[0..nl]: layer widths.  W[l]: [dims[l] x dims[l+1]] row-major (memory
 * layout of CuBiasedLinearity::mLinearity), updated in place.
 *
 * cpu_semantics=1: TNet --THREADS=1 (Platform.h:300-336; BiasedLinearity.cc:65-178):
 *     G = X^T E (float), g_b = sum_rows E (float loop); W += -lr * G; W += (-lr*wc*B) W;
 *     b += -lr * g_b.
 * cpu_semantics=0: CuBiasedLinearity::Update "#if 1" branch (cuBiasedLinearity.cc:46-64):
 *     N = (gdf ? B : 1) / (1 - mmt); C_W = X^T E + mmt C_W; c_b = colsum(E) + mmt c_b;
 *     W += (-lr/N) C_W; b += (-lr/N) c_b; W += (-lr*wc*(gdf ? 1 : B)) W.
 * Backward uses the pre-update weights (cuNetwork.h:170-194); the first layer is the stopper.
 * cW/cb (momentum buffers) are required only when cpu_semantics=0.
 * Outputs: Y (softmax output [B x nout]), E (top error [B x nout]), xent, correct (accumulated).
 * ------------------------------------------------------------------------------------- */
int orc_mlp_step(int nl, const int* dims, float** W, float** b, float** cW, float** cb,
                 const float* X, const int* lab, int B, float lr, float mmt, float wc, int gdf,
                 int cpu_semantics, float* Y, float* E, double* xent, long* correct) {
  float** act = (float**)calloc((size_t)nl + 1, sizeof(float*));   /* act[0] = X, act[l+1] = out of layer l */
  act[0] = (float*)X;
  for (int l = 0; l < nl; l++) {
    int n_in = dims[l], n_out = dims[l + 1];
    float* z = (float*)malloc(sizeof(float) * (size_t)B * n_out);
    orc_affine(act[l], B, n_in, W[l], b[l], n_out, z);
    if (l < nl - 1) orc_sigmoid(z, z, (long)B * n_out);
    else orc_softmax(z, z, B, n_out);
    act[l + 1] = z;
  }
  int nout = dims[nl];
  memcpy(Y, act[nl], sizeof(float) * (size_t)B * nout);
  float* e = (float*)malloc(sizeof(float) * (size_t)B * nout);
  orc_xent_eval(act[nl], lab, B, nout, e, xent, correct);
  memcpy(E, e, sizeof(float) * (size_t)B * nout);

  for (int l = nl - 1; l >= 0; l--) {
    int n_in = dims[l], n_out = dims[l + 1];
    float* e_in = NULL;
    if (l > 0) {  /* backprop with pre-update W, then through the sigmoid below */
      e_in = (float*)malloc(sizeof(float) * (size_t)B * n_in);
      orc_sgemm('N', 'T', B, n_in, n_out, 1.0f, e, n_out, W[l], n_out, 0.0f, e_in, n_in);
      orc_diff_sigmoid(e_in, e_in, act[l], (long)B * n_in);
    }
    size_t nw = (size_t)n_in * n_out;
    if (cpu_semantics) {
      float* G = (float*)malloc(sizeof(float) * nw);
      orc_sgemm('T', 'N', n_in, n_out, B, 1.0f, act[l], n_in, e, n_out, 0.0f, G, n_out);
      float* gb = (float*)calloc((size_t)n_out, sizeof(float));
      for (int r = 0; r < B; r++)
        for (int c = 0; c < n_out; c++) gb[c] += e[(size_t)r * n_out + c];
      for (size_t i = 0; i < nw; i++) W[l][i] = W[l][i] + (-lr) * G[i];
      float l2 = -lr * wc * (float)B;
      if (l2 != 0.0f) for (size_t i = 0; i < nw; i++) W[l][i] = W[l][i] + l2 * W[l][i];
      for (int c = 0; c < n_out; c++) b[l][c] = b[l][c] + (-lr) * gb[c];
      free(G); free(gb);
    } else {
      float N = gdf ? (float)B : 1.0f;
      N *= (float)(1.0 / (1.0 - (double)mmt));
      orc_sgemm('T', 'N', n_in, n_out, B, 1.0f, act[l], n_in, e, n_out, mmt, cW[l], n_out);
      orc_add_col_sum(1.0f, e, B, n_out, mmt, cb[l]);
      float s = -lr / N;
      for (size_t i = 0; i < nw; i++) W[l][i] = W[l][i] + s * cW[l][i];
      for (int c = 0; c < n_out; c++) b[l][c] = b[l][c] + s * cb[l][c];
      float l2 = -lr * wc * (gdf ? 1.0f : (float)B);
      if (l2 != 0.0f) for (size_t i = 0; i < nw; i++) W[l][i] = W[l][i] + l2 * W[l][i];
    }
    free(e);
    e = e_in;
  }
  for (int l = 1; l <= nl; l++) free(act[l]);
  free(act);
  return 0;
}

/* Forward only (TFeaCatCu / CuNetwork::Propagate): returns the network output Y. */
int orc_mlp_forward(int nl, const int* dims, float** W, float** b, const float* X, int B, float* Y) {
  const float* in = X;
  float* buf = NULL;
  for (int l = 0; l < nl; l++) {
    int n_in = dims[l], n_out = dims[l + 1];
    float* z = (float*)malloc(sizeof(float) * (size_t)B * n_out);
    orc_affine(in, B, n_in, W[l], b[l], n_out, z);
    if (l < nl - 1) orc_sigmoid(z, z, (long)B * n_out);
    else orc_softmax(z, z, B, n_out);
    free(buf);
    buf = z; in = z;
  }
  memcpy(Y, buf, sizeof(float) * (size_t)B * dims[nl]);
  free(buf);
  return 0;
}

/* ---------------------------------------------------------------------------------------
 * Fast writer of a gen_mlp_init-style (--gauss --negbias) .nnet text file for the CPU baseline
 * (tools/init/gen_mlp_init.py:36-68 layout: <biasedlinearity> nOut nIn / m nOut nIn / rows /
 * v nOut ...).  Random weights matter for timing: an all-zero init drives the backpropagated
 * errors of the lower layers into fp32 denormals, which makes x86 BLAS ~10x slower.
 * Box-Muller on a 64-bit LCG; 6 significant digits like the reference writer.
 * ------------------------------------------------------------------------------------- */
#include <stdio.h>
int orc_write_random_nnet(const char* path, const int* dims, int n, unsigned long long seed) {
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  unsigned long long s = seed * 6364136223846793005ull + 1442695040888963407ull;
#define ORC_U01() ((s = s * 6364136223846793005ull + 1442695040888963407ull), ((double)(s >> 11) + 0.5) / 9007199254740992.0)
  for (int l = 0; l + 1 < n; l++) {
    int ni = dims[l], no = dims[l + 1];
    fprintf(f, "<biasedlinearity> %d %d\nm %d %d\n", no, ni, no, ni);
    for (int r = 0; r < no; r++) {
      for (int c = 0; c < ni; c++) {
        double u1 = ORC_U01(), u2 = ORC_U01();
        double g = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        fprintf(f, "%g ", 0.1 * g);
      }
      fputc('\n', f);
    }
    fprintf(f, "v %d  ", no);
    for (int c = 0; c < no; c++) fprintf(f, "%g ", (l + 2 == n) ? 0.0 : ORC_U01() / 5.0 - 4.1);
    fprintf(f, "\n<%s> %d %d\n", (l + 2 == n) ? "softmax" : "sigmoid", no, no);
  }
#undef ORC_U01
  return fclose(f) == 0 ? 0 : -1;
}


/* ---------------------------------------------------------------------------------------
 * CuRand (src/CuBaseLib/curand.tcc:13-154, curandkernels.cu:14-107): per-element HybridTaus
 * state z1..z4, seeded row by row from lrand48 (values > 128), z1 first.  Arrays here are dense
 * [n] in element order.
 * ------------------------------------------------------------------------------------- */
static unsigned orc_taus(unsigned* z, int s1, int s2, int s3, unsigned m) {
  unsigned b = ((*z << s1) ^ *z) >> s2;
  return *z = ((*z & m) << s3) ^ b;
}

static float orc_hybrid_taus(unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4) {
  float r;
  do {
    unsigned x = orc_taus(z1, 13, 19, 12, 4294967294u) ^ orc_taus(z2, 2, 25, 4, 4294967288u) ^
                 orc_taus(z3, 3, 11, 17, 4294967280u) ^ (*z4 = 1664525u * *z4 + 1013904223u);
    r = (float)(2.3283064365387e-10 * (double)x);
  } while (!(r > 0.0f && r < 1.0f));
  return r;
}

static float orc_box_muller(unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4) {
  const float two_pi = 6.283185307179586476925286766558f;
  float u0 = orc_hybrid_taus(z1, z2, z3, z4), u1 = orc_hybrid_taus(z1, z2, z3, z4);
  float r = (float)sqrt(-2.0 * (double)logf(u0));
  float th = two_pi * u1;
  return r * sinf(th);
}

/* srand48(seed), then SeedGpu(rows, cols) draws; returns the lrand48 state afterwards */
uint64_t orc_rand_seed(long seed, long n, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4) {
  orc_rng48 r; orc_srand48(&r, seed);
  unsigned* zs[4] = {z1, z2, z3, z4};
  for (int k = 0; k < 4; k++)
    for (long i = 0; i < n; i++) {
      unsigned v = 0;
      while (v <= 128) v = (unsigned)orc_lrand48(&r);
      zs[k][i] = v;
    }
  return r.x;
}

void orc_rand_uniform(float* out, long n, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4) {
  for (long i = 0; i < n; i++) out[i] = orc_hybrid_taus(z1 + i, z2 + i, z3 + i, z4 + i);
}

void orc_gauss_rand(float* out, long n, unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4) {
  for (long i = 0; i < n; i++) out[i] = orc_box_muller(z1 + i, z2 + i, z3 + i, z4 + i);
}

/* One CD-1 step of the TRbmCu loop (TRbmCu.cc:329-350) with CuRbm's formulas and operation
 * order (cuRbm.cc:15-23 Propagate, :117-128 Reconstruct, :133-174 RbmUpdate):
 *   pos_hid = act(hb + pos_vis W)
 *   states  = pos_hid > U (Bernoulli hidden) | pos_hid + N(0,1) (Gaussian hidden)
 *   neg_vis = act(vb + states W^T) ; neg_hid = act(hb + neg_vis W)
 *   cW = -lr/B neg_vis^T neg_hid + mmt cW ; cW += lr/B pos_vis^T pos_hid ; cW += -lr wc W ; W += cW
 *   cvb, chb likewise from column sums ; vb += cvb ; hb += chb
 *   mse += sum (neg_vis - pos_vis)^2
 * W [V x H]; z arrays dense [B x H]; neg_vis_out [B x V] (may be NULL). */
int orc_rbm_step(int V, int H, float* W, float* vb, float* hb, float* cW, float* cvb, float* chb,
                 const float* pos_vis, int B, int vis_gauss, int hid_gauss, float lr, float mmt, float wc,
                 unsigned* z1, unsigned* z2, unsigned* z3, unsigned* z4, float* neg_vis_out, double* mse) {
  const long nh = (long)B * H, nv = (long)B * V;
  float* pos_hid = (float*)malloc(sizeof(float) * nh);
  float* states = (float*)malloc(sizeof(float) * nh);
  float* neg_vis = (float*)malloc(sizeof(float) * nv);
  float* neg_hid = (float*)malloc(sizeof(float) * nh);
  if (!pos_hid || !states || !neg_vis || !neg_hid) return -1;
  orc_affine(pos_vis, B, V, W, hb, H, pos_hid);
  if (!hid_gauss) orc_sigmoid(pos_hid, pos_hid, nh);
  if (!hid_gauss) {
    for (long i = 0; i < nh; i++) states[i] = pos_hid[i] > orc_hybrid_taus(z1 + i, z2 + i, z3 + i, z4 + i) ? 1.0f : 0.0f;
  } else {
    for (long i = 0; i < nh; i++) states[i] = 1.0f * orc_box_muller(z1 + i, z2 + i, z3 + i, z4 + i) + 1.0f * pos_hid[i];
  }
  /* neg_vis = vb + states W^T */
  for (int r = 0; r < B; r++)
    for (int c = 0; c < V; c++) neg_vis[(size_t)r * V + c] = vb[c];
  orc_sgemm('N', 'T', B, V, H, 1.0f, states, H, W, H, 1.0f, neg_vis, V);
  if (!vis_gauss) orc_sigmoid(neg_vis, neg_vis, nv);
  orc_affine(neg_vis, B, V, W, hb, H, neg_hid);
  if (!hid_gauss) orc_sigmoid(neg_hid, neg_hid, nh);
  const float N = (float)B;
  orc_sgemm('T', 'N', V, H, B, -lr / N, neg_vis, V, neg_hid, H, mmt, cW, H);
  orc_sgemm('T', 'N', V, H, B, +lr / N, pos_vis, V, pos_hid, H, 1.0f, cW, H);
  for (long i = 0; i < (long)V * H; i++) cW[i] = (-lr * wc) * W[i] + 1.0f * cW[i];
  for (long i = 0; i < (long)V * H; i++) W[i] = 1.0f * cW[i] + 1.0f * W[i];
  orc_add_col_sum(-lr / N, neg_vis, B, V, mmt, cvb);
  orc_add_col_sum(+lr / N, pos_vis, B, V, 1.0f, cvb);
  for (int i = 0; i < V; i++) vb[i] = 1.0f * cvb[i] + 1.0f * vb[i];
  orc_add_col_sum(-lr / N, neg_hid, B, H, mmt, chb);
  orc_add_col_sum(+lr / N, pos_hid, B, H, 1.0f, chb);
  for (int i = 0; i < H; i++) hb[i] = 1.0f * chb[i] + 1.0f * hb[i];
  double e2 = 0.0;
  for (long i = 0; i < nv; i++) {
    float e = neg_vis[i] - pos_vis[i];
    e2 += (double)(e * e);
  }
  if (mse) *mse += e2;
  if (neg_vis_out) memcpy(neg_vis_out, neg_vis, sizeof(float) * nv);
  free(pos_hid); free(states); free(neg_vis); free(neg_hid);
  return 0;
}

/* ---------------------------------------------------------------------------------------
 * TRecurrentCu (TRecurrentCu.cc:319-375) over [<recurrent> nIn->H, <biasedlinearity> H->S,
 * <softmax>] with cross-entropy, one utterance, frame by frame:
 *   CuRecurrent::PropagateFnc (cuRecurrent.cc:16-53): history ring push of [x_t, y_{t-1}],
 *     y_t = sigmoid(br + row Wr)
 *   CuBiasedLinearity forward + softmax; objective err = out - onehot
 *   CuNetwork::Backpropagate: <biasedlinearity> error e = err W2^T (old W2), its GPU update
 *     (cuBiasedLinearity.cc:46-64, rows = 1); <recurrent> is the stopper: Update only
 *     (cuRecurrent.cc:88-153: d_0 = e y(1-y); d_i = (Wr[nIn:] d_{i-1}) y_{t-i}(1-y_{t-i});
 *     corr = sum_i -lr h_i (x) d_i ; corr += -lr wc Wr ; Wr += corr ; bias with momentum)
 * State arrays are updated in place; hist [(bptt+1) x (nIn+H)] and y_prev [H] are zeroed here
 * (ClearHistory at the utterance start).  Returns 0.
 * ------------------------------------------------------------------------------------- */
int orc_rnn_utterance(int nIn, int H, int S, float* Wr, float* br, float* cbr, float* W2, float* b2, float* cW2,
                      float* cb2, const float* feats, const int* labels, int T, int bptt, float lr, float mmt,
                      float wc, int gdf, double* xent, long* correct) {
  const int K = nIn + H, R = bptt + 1;
  float* hist = (float*)calloc((size_t)R * K, sizeof(float));
  float* y = (float*)calloc((size_t)H, sizeof(float));
  float* out = (float*)malloc(sizeof(float) * S);
  float* err = (float*)malloc(sizeof(float) * S);
  float* e = (float*)malloc(sizeof(float) * H);
  float* D = (float*)malloc(sizeof(float) * (size_t)R * H);
  if (!hist || !y || !out || !err || !e || !D) return -1;
  int head = 0;
  for (int t = 0; t < T; t++) {
    /* forward: recurrent layer */
    head = (head + R - 1) % R;
    float* row = hist + (size_t)head * K;
    memcpy(row, feats + (size_t)t * nIn, sizeof(float) * nIn);
    memcpy(row + nIn, y, sizeof(float) * H);
    for (int c = 0; c < H; c++) {
      double s = br[c];
      for (int k = 0; k < K; k++) s += (double)row[k] * Wr[(size_t)k * H + c];
      y[c] = (float)(1.0 / (1.0 + exp(-(double)(float)s)));
    }
    /* output layer + softmax + objective */
    float* a = out;
    for (int c = 0; c < S; c++) {
      double s = b2[c];
      for (int k = 0; k < H; k++) s += (double)y[k] * W2[(size_t)k * S + c];
      a[c] = (float)s;
    }
    orc_softmax(out, a, 1, S);
    orc_xent_eval(out, labels + t, 1, S, err, xent, correct);
    /* <biasedlinearity>: backpropagate with the old weights, then its GPU update (rows = 1) */
    for (int k = 0; k < H; k++) {
      double s = 0.0;
      for (int c = 0; c < S; c++) s += (double)err[c] * W2[(size_t)k * S + c];
      e[k] = (float)s;
    }
    {
      float N = 1.0f;  /* GRADDIVFRM: rows = 1 either way */
      (void)gdf;
      N *= (float)(1.0 / (1.0 - mmt));
      const float scale = -lr / N, l2 = -lr * wc;
      for (int k = 0; k < H; k++)
        for (int c = 0; c < S; c++) {
          float* cp = cW2 + (size_t)k * S + c;
          float* wp = W2 + (size_t)k * S + c;
          *cp = y[k] * err[c] + mmt * *cp;
          float w = *wp + scale * *cp;
          *wp = w + l2 * w;
        }
      for (int c = 0; c < S; c++) {
        cb2[c] = err[c] + mmt * cb2[c];
        b2[c] = b2[c] + scale * cb2[c];
      }
    }
    /* <recurrent> update with BPTT */
    for (int c = 0; c < H; c++) D[c] = (float)((double)y[c] * (1.0 - (double)y[c]) * (double)e[c]);
    for (int i = 1; i <= bptt; i++) {
      const float* hy = hist + (size_t)((head + i - 1) % R) * K + nIn;
      for (int r = 0; r < H; r++) {
        double s = 0.0;
        for (int c = 0; c < H; c++) s += (double)Wr[(size_t)(nIn + r) * H + c] * D[(size_t)(i - 1) * H + c];
        D[(size_t)i * H + r] = (float)((float)s * (hy[r] * (1.0f - hy[r])));
      }
    }
    for (int k = 0; k < K; k++)
      for (int c = 0; c < H; c++) {
        float acc = 0.f;
        for (int i = 0; i < R; i++) acc += (-lr * hist[(size_t)((head + i) % R) * K + k]) * D[(size_t)i * H + c];
        float* wp = Wr + (size_t)k * H + c;
        const float w = *wp;
        *wp = ((-lr * wc) * w + acc) + w;
      }
    for (int c = 0; c < H; c++) {
      float g = -lr * D[c] + mmt * cbr[c];
      for (int i = 1; i < R; i++) g = -lr * D[(size_t)i * H + c] + g;
      cbr[c] = g;
      br[c] = g + br[c];
    }
  }
  free(hist); free(y); free(out); free(err); free(e); free(D);
  return 0;
}
