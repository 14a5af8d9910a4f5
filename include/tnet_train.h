/*
 * tnet_train.h -- C ABI of the MI355X TNet training library (libtnet_amd.so), above the kernels.
 *
 * The reference exposes this layer as C++ classes only; these entry points are what an FFI
 * (ctypes / cgo / JNI) binding of the CuComponent / CuNetwork / CuObjectiveFunction / CuCache /
 * TNetCu-loop API binds to.  Each function names the reference interface it replaces.
 * The C++ classes themselves (nnet-asr_amd/csrc/host/ headers) keep the reference names for C++ users.
 *
 * Conventions: opaque handles; device pointers are raw HIP device memory (see tnet_malloc);
 * host pointers are plain arrays; all row-major with explicit leading dimensions (elements).
 * Return 0 on success, a negative status on failure; tnet_last_error() gives the message of the
 * last failure on the calling thread (the reference throws MyException, src/KaldiLib/Error.h).
 */
#ifndef TNET_TRAIN_H_
#define TNET_TRAIN_H_

#include <stddef.h>

#include "tnet_kernels.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct TnetNetwork TnetNetwork;
typedef struct TnetObjective TnetObjective;
typedef struct TnetTrainer TnetTrainer;
typedef struct TnetComm TnetComm;
typedef struct TnetRbmTrainer TnetRbmTrainer;
typedef struct TnetRnnTrainer TnetRnnTrainer;

const char* tnet_last_error(void);

/* ---- runtime (CuDevice, src/CuBaseLib/cudevice.h:15-73) ------------------------------ */
int tnet_device_count(int* n);
int tnet_select_gpu(int gpu_id);               /* CuDevice::SelectGPU (cudevice.cc:84-101) */
int tnet_synchronize(void);                    /* drain the library stream */
void* tnet_stream(void);                       /* the library's hipStream_t */
int tnet_malloc(void** p, size_t bytes);
int tnet_free(void* p);
int tnet_memcpy_h2d(void* dst, const void* src, size_t bytes);
int tnet_memcpy_d2h(void* dst, const void* src, size_t bytes);
int tnet_memcpy_d2d(void* dst, const void* src, size_t bytes);
int tnet_memset(void* dst, int value, size_t bytes);
int tnet_set_profile(int on);                  /* CuDevice::Verbose + AccuProfile map */
int tnet_profile_report(char* buf, int cap);
/* Per-kernel device timing (hipEvent pairs on the library stream).  on = 1: a pair around each timed
 * launch; on = 2: one pair per RUN of consecutive timed launches (a launch whose tag fails the filter
 * ends the run), the run's time split over its tags by work share and the exact run totals on a
 * "@runs:<n> launches total_ms total_work" line.  The report lists "tag count total_ms total_work"
 * lines (work = algorithmic FLOPs for GEMMs, bytes for HBM-bound kernels) since the last report. */
int tnet_kernel_timing(int on);
/* time only launches whose tag contains `filter` ("" or NULL = all), e.g. ":2048x2048" */
int tnet_kernel_timing_filter(const char* filter);
int tnet_kernel_timing_report(char* buf, int cap);
/* Device-side timing of the enqueued work: start/stop return elapsed ms between two marks. */
int tnet_timer_start(void);
int tnet_timer_stop(float* ms);

/* ---- network (CuNetwork, src/CuTNetLib/cuNetwork.h:22-194) ---------------------------- */
TnetNetwork* tnet_net_read(const char* path);  /* ReadNetwork(const char*)   (cuNetwork.cc:27-37) */
TnetNetwork* tnet_net_read_text(const char* text); /* ReadNetwork(istream&)  (cuNetwork.cc:53-61) */
int tnet_net_write(TnetNetwork* net, const char* path); /* WriteNetwork       (cuNetwork.cc:40-50) */
int tnet_net_free(TnetNetwork* net);
int tnet_net_num_components(TnetNetwork* net);  /* Layers() */
/* Layer(i): tag (GetName), inputs/outputs (GetNInputs/GetNOutputs) */
int tnet_net_component(TnetNetwork* net, int i, char* tag, int cap, int* n_in, int* n_out);
/* <biasedlinearity> parameters in memory layout: W [n_in x n_out] row-major, b [n_out] (host) */
int tnet_net_get_params(TnetNetwork* net, int i, float* W, float* b);
int tnet_net_set_params(TnetNetwork* net, int i, const float* W, const float* b);
int tnet_net_set_learn_rate(TnetNetwork* net, float lr, const char* factors); /* SetLearnRate (cuNetwork.cc:80-134) */
int tnet_net_set_momentum(TnetNetwork* net, float mmt);                       /* SetMomentum */
int tnet_net_set_weightcost(TnetNetwork* net, float wc);                      /* SetWeightcost */
int tnet_net_set_grad_div_frm(TnetNetwork* net, int div);                     /* SetGradDivFrm */
/* Propagate (cuNetwork.h:137-165): X [rows x n_in] -> Y [rows x n_out], device pointers */
int tnet_net_propagate(TnetNetwork* net, const float* dX, int rows, int ldx, float* dY, int ldy);
/* Backpropagate (cuNetwork.h:170-194): global error [rows x n_out] of the LAST Propagate */
int tnet_net_backpropagate(TnetNetwork* net, const float* dE, int rows, int lde);
/* One fused SGD step (MI355X path): Propagate + CuCrossEntropy::Evaluate + Backpropagate with
 * class-id targets (label < 0 = unlabeled frame); train = 0 -> forward + objective only */
int tnet_net_train_bunch(TnetNetwork* net, TnetObjective* obj, const float* dX, int rows, int ldx,
                         const int* dLabels, int train);
/* Keep the softmax output of tnet_net_train_bunch readable via tnet_net_output (extra write) */
int tnet_net_keep_output(TnetNetwork* net, int keep);
/* output of component i (GetOutput) copied to host [rows x n_out] */
int tnet_net_output(TnetNetwork* net, int i, float* host, int ld);

/* ---- objective (CuObjectiveFunction, src/CuTNetLib/cuObjectiveFunction.h:20-157) ----- */
TnetObjective* tnet_obj_create(int type);      /* 0 = CROSS_ENTROPY (xent), 1 = MEAN_SQUARE_ERROR (mse) */
int tnet_obj_free(TnetObjective* obj);
/* Evaluate(out, desired, err) with a dense desired matrix (cuObjectiveFunction.cc:28-83) */
int tnet_obj_evaluate(TnetObjective* obj, const float* dOut, int rows, int cols, int ldo, const float* dDes,
                      int ldd, float* dErr, int lde);
/* class-id targets */
int tnet_obj_evaluate_labels(TnetObjective* obj, const float* dOut, int rows, int cols, int ldo,
                             const int* dLabels, float* dErr, int lde);
/* GetError / GetFrames / correct count */
int tnet_obj_stats(TnetObjective* obj, double* error, long* frames, double* correct);
/* Report() line, e.g. "Xent:187469 frames:54720 err/frm:3.42598 correct[23.2365%]\n" */
int tnet_obj_report(TnetObjective* obj, char* buf, int cap);
int tnet_obj_reset(TnetObjective* obj);

/* ---- trainer: the TNetCu SGD loop (src/TNetCu.cc:375-442) + CuCache (cuCache.h:12-70) ----- */
TnetTrainer* tnet_trainer_create(TnetNetwork* net, TnetObjective* obj, int bunchsize, int cachesize, long seed,
                                 int randomize, int crossval);
int tnet_trainer_free(TnetTrainer* t);
/* one utterance in scp order: features [rows x cols] (ld), class ids [rows] (host memory) */
int tnet_trainer_add_utterance(TnetTrainer* t, const float* feats, int rows, int cols, int ld, const int* labels);
int tnet_trainer_finish(TnetTrainer* t);       /* EndOfList */
long tnet_trainer_steps(TnetTrainer* t);
int tnet_trainer_replay(TnetTrainer* t, long nsteps); /* benchmark: more steps over the resident cache */
/* benchmark setup: load host frames into the cache without training; returns rows taken (<0 error) */
long tnet_trainer_prefill(TnetTrainer* t, const float* feats, int rows, int cols, int ld, const int* labels);
/* fault injection (tests): the n-th next network training step throws before it enqueues anything (the
   call that ran it returns TNET_ERR_RUNTIME); 0 disarms.  No reference counterpart (test hook). */
int tnet_debug_fail_train_bunch(long n);
int tnet_trainer_set_comm(TnetTrainer* t, TnetComm* comm);
/* data-parallel steps this rank joined without a bunch of its own (zero gradient) */
long tnet_trainer_empty_steps(TnetTrainer* t);
int tnet_trainer_trace(TnetTrainer* t, int trace);
/* --FEATURETRANSFORM / --STARTFRMEXT / --ENDFRMEXT (TNetCu.cc:274-278, 384-393): each utterance
 * passed to add_utterance is edge-extended, propagated through `transform` (a front-end network,
 * borrowed, may be NULL = off) and trimmed before the cache; labels stay one per input frame */
int tnet_trainer_set_transform(TnetTrainer* t, TnetNetwork* transform, int start_ext, int end_ext);

/* ---- host front end: HTK features + MLF targets, read ahead by a thread pool -----------------
 * Replaces FeatureRepository (src/KaldiLib/Features.cc:349-477, 1009-1347: Init / AddFileList /
 * ReadFullMatrix / MoveNext with STARTFRMEXT / ENDFRMEXT, TARGETKIND, NATURALREADORDER) and
 * LabelRepository (src/KaldiLib/Labels.cc:11-186: Init / GenDesiredMatrix, as class ids), the
 * intake TNetCu drives at TNetCu.cc:290-314, 376-419.  Pure host code (no device calls).
 *   swap         : byte-swap the big-endian HTK data (!NATURALREADORDER on this host: 1)
 *   target_kind  : HTK parameter kind, 12 = ANON (the first file's kind); deriv_order as DERIVWINDOWS
 *                  (0 with ANON: derivatives in the file are dropped, as the reference; < 0: the
 *                  first file's); deriv_win: NULL or deriv_order window lengths (default 2 each)
 *   mlf == NULL  : features only (labels / n_labels come back NULL / 0)
 *   label_dir / label_ext : SOURCETRANSCDIR / SOURCETRANSCEXT (NULL / "lab" in TNetCu)
 *   threads, depth : reader threads and utterances read ahead of the consumer */
typedef struct TnetFeatureReader TnetFeatureReader;
TnetFeatureReader* tnet_reader_create(const char* scp, int swap, int start_ext, int end_ext, int target_kind,
                                      int deriv_order, const int* deriv_win, const char* mlf, const char* label_map,
                                      const char* label_dir, const char* label_ext, int threads, int depth);
/* the same with cepstral mean / variance normalisation (Features.cc:1352-1410, the TNetCu keys CMEANDIR,
 * CMEANMASK, VARSCALEDIR, VARSCALEMASK, VARSCALEFN; UserInterface.cc:385-410): a NULL mask (file) turns that
 * step off; the mean / variance file of an utterance is <dir>/ + "/" + the characters the mask's '%'s
 * capture from its logical name */
TnetFeatureReader* tnet_reader_create_norm(const char* scp, int swap, int start_ext, int end_ext, int target_kind,
                                           int deriv_order, const int* deriv_win, const char* mlf,
                                           const char* label_map, const char* label_dir, const char* label_ext,
                                           const char* cmn_dir, const char* cmn_mask, const char* cvn_dir,
                                           const char* cvn_mask, const char* cvg_file, int threads, int depth);
int tnet_reader_free(TnetFeatureReader* r);
long tnet_reader_size(TnetFeatureReader* r);  /* records in the script */
/* next utterance in script order: 1 = delivered, 0 = end of list, < 0 = this record's error (the
 * reference's exception text in tnet_last_error).  feats [rows x cols] dense row-major incl. the
 * context rows; labels [n_labels = rows - start_ext - end_ext]; pointers valid until the next call. */
int tnet_reader_next(TnetFeatureReader* r, const float** feats, int* rows, int* cols, const int** labels,
                     int* n_labels, int* samp_period, int* kind, char* logical, int logical_cap);
int tnet_reader_rewind(TnetFeatureReader* r);  /* FeatureRepository::Rewind */
/* one record ("logical=physical[s,e]" or a path) without a reader: out == NULL asks for the size only */
int tnet_htk_read(const char* record, int swap, int start_ext, int end_ext, float* out, long cap, int* rows, int* cols,
                  int* samp_period, int* kind);
/* label masks and the MLF record index on their own (csrc/host/labelindex.h):
 *   tnet_mask_match: ProcessMask (src/KaldiLib/StkMatch.cc:453-490) -- 1 when `mask`, anchored at a path
 *     component, matches `label`, with the characters its '%'s capture in captured[cap] (NUL-terminated,
 *     truncated to cap); 0 when it does not; < 0 on an argument error
 *   tnet_mlf_lookup: LabelContainer::Insert of patterns[k] as record k, k = 0..n_patterns-1, in order
 *     (MlfStream.cc:43-93), then LabelContainer::Find of each label (MlfStream.cc:243-262): rec_out[i] = the
 *     record label i resolves to, -1 for none */
int tnet_mask_match(const char* mask, const char* label, char* captured, int cap);
int tnet_mlf_lookup(const char* const* patterns, int n_patterns, const char* const* labels, int n_labels,
                    int* rec_out);
/* the cache fill of TNetCu.cc:376-419 from a reader: up to max_utts utterances (< 0: to the end of the
 * list) into the trainer, each training the cache whenever it fills; returns the frames added (< 0 error).
 * The reader's STARTFRMEXT / ENDFRMEXT must be the transform's (tnet_trainer_set_transform); without
 * a transform the context rows are trimmed.  An utterance holding a NaN / Inf is rejected with
 * TNetCu's CheckData error (TNetCu.cc:386), as the reference driver does. */
long tnet_trainer_add_reader(TnetTrainer* t, TnetFeatureReader* r, long max_utts);

/* ---- RBM pre-training (CuRbm, cuRbm.cc; the TRbmCu loop, TRbmCu.cc:291-357) ----------------
 * <rbm> parameters: W [n_vis x n_hid] (host row-major), visible / hidden biases; types[0..1] =
 * visible / hidden unit type (0 Bernoulli, 1 Gaussian; -1 in set = keep). */
int tnet_net_rbm_get(TnetNetwork* net, int i, float* W, float* vis_bias, float* hid_bias, int* types);
int tnet_net_rbm_set(TnetNetwork* net, int i, const float* W, const float* vis_bias, const float* hid_bias,
                     int vis_type, int hid_type);
/* CuRbm::RbmUpdate on four device matrices [rows x n_vis|n_hid] (cuRbm.cc:133-174) */
int tnet_net_rbm_update(TnetNetwork* net, int i, const float* pos_vis, const float* pos_hid, const float* neg_vis,
                        const float* neg_hid, int rows, int ld_vis, int ld_hid);
/* CD-1 trainer over a one-<rbm> network (TRbmCu): per bunch positive phase, sample (Bernoulli)
 * or Gaussian noise, reconstruct, negative phase, update, reconstruction MSE. seed as TRbmCu
 * --SEED (CuRand state drawn first, then the cache shuffles, one lrand48 stream). */
TnetRbmTrainer* tnet_rbm_trainer_create(TnetNetwork* net, int bunchsize, int cachesize, long seed, int randomize,
                                        float learn_rate, float momentum, float weightcost);
int tnet_rbm_trainer_free(TnetRbmTrainer* t);
int tnet_rbm_trainer_add_utterance(TnetRbmTrainer* t, const float* feats, int rows, int cols, int ld);
int tnet_rbm_trainer_finish(TnetRbmTrainer* t);
long tnet_rbm_trainer_steps(TnetRbmTrainer* t);
int tnet_rbm_trainer_stats(TnetRbmTrainer* t, double* mse, long* frames);
int tnet_rbm_trainer_report(TnetRbmTrainer* t, char* buf, int cap); /* "Mse:... frames:... err/frm:..." */
long tnet_rbm_trainer_prefill(TnetRbmTrainer* t, const float* feats, int rows, int cols, int ld);
int tnet_rbm_trainer_replay(TnetRbmTrainer* t, long nsteps);

/* ---- recurrent training (CuRecurrent, cuRecurrent.cc; the TRecurrentCu loop, TRecurrentCu.cc:319-375) --
 * <recurrent> parameters: W [(n_in + n_out) x n_out] (host row-major), bias [n_out]. */
int tnet_net_recurrent_get(TnetNetwork* net, int i, float* W, float* b);
int tnet_net_recurrent_set(TnetNetwork* net, int i, const float* W, const float* b);
/* Frame-by-frame trainer: sets the BPTT order of every <recurrent> layer (--BPTT); per utterance
 * clears the history, then per frame propagate / objective / backpropagate+update. */
TnetRnnTrainer* tnet_rnn_trainer_create(TnetNetwork* net, TnetObjective* obj, int bptt, int crossval);
int tnet_rnn_trainer_free(TnetRnnTrainer* t);
int tnet_rnn_trainer_utterance(TnetRnnTrainer* t, const float* feats, int rows, int cols, int ld, const int* labels);
long tnet_rnn_trainer_frames(TnetRnnTrainer* t);

/* ---- data parallel (no reference counterpart: Platform.h:143-391 is the CPU analogue) ---- */
int tnet_comm_unique_id(char out[128]);        /* rank 0 creates, the launcher broadcasts it */
TnetComm* tnet_comm_create(int rank, int world, const char id[128]);
int tnet_comm_free(TnetComm* comm);
int tnet_comm_allreduce_host(TnetComm* comm, double* v, int n);
int tnet_comm_allreduce_device(TnetComm* comm, float* dbuf, long n);
/* the reduction check (bench.py rccl_check; the reference's reduce is Platform.h:307-335): tnet_comm_capture(comm, 1)
 * arms ONE step -- every gradient block the next step submits is copied to the host right before its reduction
 * (this rank's local gradient) and right after it (the reduced values over the ranges this rank applies, NaN
 * elsewhere); synchronous, for a check step outside the timed region.  The copies stay until the next arming:
 * tnet_comm_captured = block count, tnet_comm_captured_block(i) fills local / reduced [n] (both NULL: n only).
 * tnet_comm_transport_ranks: the rank count as the transport reports it (ncclCommCount for RCCL). */
int tnet_comm_capture(TnetComm* comm, int on);
long tnet_comm_captured(TnetComm* comm);
int tnet_comm_captured_block(TnetComm* comm, long i, float* local, float* reduced, long cap, long* n);
int tnet_comm_transport_ranks(TnetComm* comm, int* ranks);
/* Host-transport communicator: gradients are staged through host memory and summed in place by
 * fn(user, buf, n, is_double) (float32 when is_double == 0); fn returns 0 on success.  For
 * transports without RCCL (gloo, MPI) and multi-process tests on one device; PCIe-bound. */
typedef int (*tnet_host_allreduce_fn)(void* user, void* buf, long n, int is_double);
TnetComm* tnet_comm_create_host(int rank, int world, tnet_host_allreduce_fn fn, void* user);
/* One round of the data-parallel step plan (collective over the communicator): this rank holds
 * n bunches, final != 0 if it has reached the end of its utterances.  Returns the round's step
 * count, the number of ranks holding a bunch at each step (ranks_at_step[cap]) and whether all
 * ranks are final.  Pure host logic. */
int tnet_dp_plan_round(TnetComm* comm, long n, int final, long* steps, int* ranks_at_step, long cap,
                       int* all_final);
/* The sharded apply's split of an n-element parameter block over `world` ranks (what the RCCL
 * communicator reduce-scatters / all-gathers; a maintainer's own transport needs the same split):
 * rank r updates [lo[k], hi[k]) for k < *count (<= 2): its shard [r c, (r + 1) c), c a multiple of
 * 4 elements, and the tail [world c, n) that every rank updates.  Pure host logic. */
int tnet_dp_shard_ranges(long n, int rank, int world, long* lo, long* hi, int* count);
/* Network-level data parallelism: tnet_net_train_bunch all-reduces the weight gradients over
 * comm (NULL = local update); a rank without a bunch calls tnet_net_train_empty with the global
 * row count of the step. */
int tnet_net_set_comm(TnetNetwork* net, TnetComm* comm);
/* Rows of the global bunch of the next steps (GRADDIVFRM normalisation) when the ranks' bunches
 * differ in size; 0 restores the default local rows x world size. */
int tnet_comm_set_step_rows(TnetComm* comm, long global_rows);
int tnet_net_train_empty(TnetNetwork* net, TnetComm* comm, long global_rows);

#ifdef __cplusplus
}
#endif
#endif /* TNET_TRAIN_H_ */
