"""ctypes binding of lib/libtnet_amd.so (include/tnet_kernels.h + include/tnet_train.h).

This is the reference-side binding INTEGRATION.md describes: plain C ABI, raw pointers, sizes,
status codes.  Loading the library never touches the GPU; the first call that needs the device
does.  There is no fallback: if the shared library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libtnet_amd.so")
if os.environ.get("TNET_DIAG_STAMP_LIB"):  # diagnostics only (tools/gemm_clock.py): clock-stamped GEMM build
    _v = os.environ["TNET_DIAG_STAMP_LIB"]
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libtnet_amd_stamp" + ("" if _v == "1" else "_" + _v) + ".so")
if os.environ.get("TNET_LIB_VARIANT"):  # diagnostics only: e.g. "precise" (make -C nnet-asr_amd precise)
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libtnet_amd_" + os.environ["TNET_LIB_VARIANT"] + ".so")
INCLUDE_DIR = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include")

_lib = None


class TnetError(RuntimeError):
    pass


class MatrixDim(C.Structure):
    _fields_ = [("rows", C.c_int), ("cols", C.c_int), ("stride", C.c_int)]


vp = C.c_void_p
i32 = C.c_int
f32 = C.c_float
i64 = C.c_long
dp = C.POINTER(C.c_double)

# name -> (restype, argtypes)
_SIGS = {
    # tnet_kernels.h
    "tnet_status_str": (C.c_char_p, [i32]),
    "tnet_version": (C.c_char_p, []),
    "tnetF_set_const": (i32, [vp, f32, MatrixDim, vp]),
    "tnetF_apply_log": (i32, [vp, MatrixDim, vp]),
    "tnetF_apply_mask": (i32, [vp, vp, MatrixDim, MatrixDim, vp]),
    "tnetF_apply_l1": (i32, [vp, f32, MatrixDim, vp]),
    "tnetF_scale_cols": (i32, [vp, vp, MatrixDim, vp]),
    "tnetF_scale_rows": (i32, [vp, vp, MatrixDim, vp]),
    "tnetF_add_scaled": (i32, [f32, vp, i32, f32, vp, MatrixDim, vp]),
    "tnetF_add_scaled_row": (i32, [f32, vp, f32, vp, MatrixDim, vp]),
    "tnetF_mul_elem": (i32, [vp, vp, i32, MatrixDim, vp]),
    "tnetF_log_elem": (i32, [vp, MatrixDim, vp]),
    "tnet_col_sum_workspace": (i64, [MatrixDim]),
    "tnetF_add_col_sum": (i32, [f32, vp, f32, vp, MatrixDim, vp, vp]),
    "tnetF_sigmoid": (i32, [vp, vp, MatrixDim, vp]),
    "tnetF_diff_sigmoid": (i32, [vp, vp, vp, MatrixDim, vp]),
    "tnetF_softmax": (i32, [vp, vp, MatrixDim, vp]),
    "tnetF_check_class": (i32, [vp, vp, vp, MatrixDim, vp]),
    "tnetF_expand": (i32, [vp, vp, vp, MatrixDim, MatrixDim, vp]),
    "tnetF_rearrange": (i32, [vp, vp, vp, MatrixDim, MatrixDim, vp]),
    "tnetF_randomize": (i32, [vp, vp, vp, MatrixDim, MatrixDim, vp]),
    "tnet_block_linearity": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp]),
    "tnet_gather_i32": (i32, [vp, vp, vp, i32, vp]),
    "tnet_gather_bunch": (i32, [vp, vp, vp, vp, vp, MatrixDim, MatrixDim, vp]),
    "tnet_sgemm": (i32, [C.c_char, C.c_char, i32, i32, i32, f32, vp, i32, vp, i32, f32, vp, i32, vp]),
    "tnet_gemm_config": (i32, [C.c_char_p]),
    "tnet_gemm_reserve": (i32, [i32]),
    "tnet_affine_fwd": (i32, [vp, MatrixDim, vp, MatrixDim, vp, vp, MatrixDim, i32, vp]),
    "tnet_affine_fwd_sample": (i32, [vp, MatrixDim, vp, MatrixDim, vp, vp, MatrixDim, vp, i32, vp, vp, vp, vp, vp]),
    "tnet_affine_bwd": (i32, [vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, i32, vp]),
    "tnet_affine_update": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp]),
    "tnet_colsum_slabs": (i32, [i32]),
    "tnet_affine_update_row": (i32, [vp, i32, vp, i32, vp, i32, vp, i32, vp, vp, f32, f32, f32, vp]),
    "tnet_affine_bwd_update_row": (i32, [vp, i32, vp, i32, vp, i32, vp, i32, vp, vp, f32, f32, f32, vp, vp, vp, vp]),
    "tnet_gemv_rowvec_cat": (i32, [vp, i32, vp, i32, vp, vp, i32, vp, vp, i32, i32, vp, vp]),
    "tnet_gemv_rowvec_softmax_xent": (i32, [vp, i32, vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp]),
    "tnet_colsum_slab_sums": (i32, [vp, MatrixDim, vp, i32, vp]),
    "tnet_affine_softmax_xent": (i32, [vp, MatrixDim, vp, MatrixDim, vp, vp, vp, i32, vp, i32, vp, i32, vp, vp, i32,
                                       vp]),
    "tnet_affine_grad_bias": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, vp, vp]),
    "tnet_affine_grad_bwd_pair": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, vp, vp, MatrixDim, vp,
                                        MatrixDim, vp, i32, vp, MatrixDim, vp, i32, vp]),
    "tnet_affine_grad_bias_gather": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, vp, vp, MatrixDim, vp,
                                           MatrixDim, vp, MatrixDim, vp, i32, vp, vp, vp, vp, vp, vp, MatrixDim,
                                           MatrixDim, vp]),
    "tnet_sgd_update_multi": (i32, [vp, i32, f32, f32, vp]),
    "tnet_affine_bwd_colsum": (i32, [vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, vp, i32, vp]),
    "tnet_affine_bwd_colsum_slabs": (i32, [vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, vp, i32, vp, i32,
                                           vp]),
    "tnet_affine_bwd_colsum_t": (i32, [vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, vp, i32, vp]),
    "tnet_affine_bwd_colsum_slabs_t": (i32, [vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, vp, i32, vp, i32,
                                             vp]),
    "tnet_affine_update_bwd_pair_t": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp,
                                            i32, vp, vp, vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, vp, i32,
                                            vp]),
    "tnet_weight_shadow": (i32, [vp, MatrixDim, vp, i32]),
    "tnet_weight_shadow_kept": (i32, [vp]),
    "tnet_transpose": (i32, [vp, MatrixDim, vp, i32, vp]),
    "tnet_affine_update_bias": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp, i32,
                                      vp, vp, vp]),
    "tnet_affine_update_bias_pair": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp, i32,
                                           vp, vp, vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32,
                                           f32, vp, i32, vp, vp, vp]),
    "tnet_affine_update_bias_gather": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp,
                                             i32, vp, vp, vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32,
                                             f32, f32, vp, i32, vp, vp, vp, vp, vp, vp, vp, MatrixDim, MatrixDim, vp]),
    "tnet_affine_update_bwd_pair": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp, i32,
                                          vp, vp, vp, MatrixDim, vp, MatrixDim, vp, i32, vp, MatrixDim, vp, i32, vp]),
    "tnet_affine_grad": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp]),
    "tnet_sgd_update": (i32, [vp, vp, vp, i64, f32, f32, f32, vp]),
    "tnet_bias_update": (i32, [vp, MatrixDim, vp, vp, vp, f32, f32, vp, vp]),
    "tnet_softmax_xent": (i32, [vp, MatrixDim, vp, vp, i32, vp, i32, vp, vp]),
    "tnet_softmax_xent_dense": (i32, [vp, MatrixDim, vp, i32, vp, i32, vp, i32, vp, vp]),
    "tnet_mse": (i32, [vp, MatrixDim, vp, i32, vp, i32, vp, vp]),
    "tnet_stats_fetch": (i32, [vp, dp, dp, vp]),
    # tnet_train.h
    "tnet_last_error": (C.c_char_p, []),
    "tnet_device_count": (i32, [C.POINTER(i32)]),
    "tnet_select_gpu": (i32, [i32]),
    "tnet_synchronize": (i32, []),
    "tnet_stream": (vp, []),
    "tnet_malloc": (i32, [C.POINTER(vp), C.c_size_t]),
    "tnet_free": (i32, [vp]),
    "tnet_memcpy_h2d": (i32, [vp, vp, C.c_size_t]),
    "tnet_memcpy_d2h": (i32, [vp, vp, C.c_size_t]),
    "tnet_memcpy_d2d": (i32, [vp, vp, C.c_size_t]),
    "tnet_memset": (i32, [vp, i32, C.c_size_t]),
    "tnet_set_profile": (i32, [i32]),
    "tnet_profile_report": (i32, [C.c_char_p, i32]),
    "tnet_kernel_timing": (i32, [i32]),
    "tnet_kernel_timing_filter": (i32, [C.c_char_p]),
    "tnet_kernel_timing_report": (i32, [C.c_char_p, i32]),
    "tnet_timer_start": (i32, []),
    "tnet_timer_stop": (i32, [C.POINTER(f32)]),
    "tnet_net_read": (vp, [C.c_char_p]),
    "tnet_net_read_text": (vp, [C.c_char_p]),
    "tnet_net_write": (i32, [vp, C.c_char_p]),
    "tnet_net_free": (i32, [vp]),
    "tnet_net_num_components": (i32, [vp]),
    "tnet_net_component": (i32, [vp, i32, C.c_char_p, i32, C.POINTER(i32), C.POINTER(i32)]),
    "tnet_net_get_params": (i32, [vp, i32, vp, vp]),
    "tnet_net_set_params": (i32, [vp, i32, vp, vp]),
    "tnet_net_set_learn_rate": (i32, [vp, f32, C.c_char_p]),
    "tnet_net_set_momentum": (i32, [vp, f32]),
    "tnet_net_set_weightcost": (i32, [vp, f32]),
    "tnet_net_set_grad_div_frm": (i32, [vp, i32]),
    "tnet_net_propagate": (i32, [vp, vp, i32, i32, vp, i32]),
    "tnet_net_backpropagate": (i32, [vp, vp, i32, i32]),
    "tnet_net_train_bunch": (i32, [vp, vp, vp, i32, i32, vp, i32]),
    "tnet_net_keep_output": (i32, [vp, i32]),
    "tnet_net_output": (i32, [vp, i32, vp, i32]),
    "tnet_obj_create": (vp, [i32]),
    "tnet_obj_free": (i32, [vp]),
    "tnet_obj_evaluate": (i32, [vp, vp, i32, i32, i32, vp, i32, vp, i32]),
    "tnet_obj_evaluate_labels": (i32, [vp, vp, i32, i32, i32, vp, vp, i32]),
    "tnet_obj_stats": (i32, [vp, dp, C.POINTER(i64), dp]),
    "tnet_obj_report": (i32, [vp, C.c_char_p, i32]),
    "tnet_obj_reset": (i32, [vp]),
    "tnet_trainer_create": (vp, [vp, vp, i32, i32, i64, i32, i32]),
    "tnet_trainer_free": (i32, [vp]),
    "tnet_trainer_add_utterance": (i32, [vp, vp, i32, i32, i32, vp]),
    "tnet_trainer_finish": (i32, [vp]),
    "tnet_trainer_steps": (i64, [vp]),
    "tnet_trainer_replay": (i32, [vp, i64]),
    "tnet_trainer_prefill": (i64, [vp, vp, i32, i32, i32, vp]),
    "tnet_debug_fail_train_bunch": (i32, [i64]),
    "tnet_trainer_set_comm": (i32, [vp, vp]),
    "tnet_trainer_trace": (i32, [vp, i32]),
    "tnet_trainer_set_transform": (i32, [vp, vp, i32, i32]),
    "tnet_reader_create": (vp, [C.c_char_p, i32, i32, i32, i32, i32, vp, C.c_char_p, C.c_char_p, C.c_char_p,
                                C.c_char_p, i32, i32]),
    "tnet_reader_create_norm": (vp, [C.c_char_p, i32, i32, i32, i32, i32, vp, C.c_char_p, C.c_char_p, C.c_char_p,
                                     C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, i32,
                                     i32]),
    "tnet_reader_free": (i32, [vp]),
    "tnet_reader_size": (i64, [vp]),
    "tnet_reader_next": (i32, [vp, C.POINTER(vp), C.POINTER(i32), C.POINTER(i32), C.POINTER(vp), C.POINTER(i32),
                              C.POINTER(i32), C.POINTER(i32), C.c_char_p, i32]),
    "tnet_reader_rewind": (i32, [vp]),
    "tnet_htk_read": (i32, [C.c_char_p, i32, i32, i32, vp, i64, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                           C.POINTER(i32)]),
    "tnet_mask_match": (i32, [C.c_char_p, C.c_char_p, C.c_char_p, i32]),
    "tnet_mlf_lookup": (i32, [vp, i32, vp, i32, vp]),
    "tnet_trainer_add_reader": (i64, [vp, vp, i64]),
    "tnet_comm_unique_id": (i32, [C.c_char_p]),
    "tnet_comm_create": (vp, [i32, i32, C.c_char_p]),
    "tnet_comm_free": (i32, [vp]),
    "tnet_comm_allreduce_host": (i32, [vp, dp, i32]),
    "tnet_comm_allreduce_device": (i32, [vp, vp, i64]),
    "tnet_comm_capture": (i32, [vp, i32]),
    "tnet_comm_captured": (i64, [vp]),
    "tnet_comm_captured_block": (i32, [vp, i64, vp, vp, i64, C.POINTER(i64)]),
    "tnet_comm_transport_ranks": (i32, [vp, C.POINTER(i32)]),
    "tnet_comm_create_host": (vp, [i32, i32, vp, vp]),
    "tnet_net_rbm_get": (i32, [vp, i32, vp, vp, vp, vp]),
    "tnet_net_rbm_set": (i32, [vp, i32, vp, vp, vp, i32, i32]),
    "tnet_net_rbm_update": (i32, [vp, i32, vp, vp, vp, vp, i32, i32, i32]),
    "tnet_rbm_trainer_create": (vp, [vp, i32, i32, i64, i32, f32, f32, f32]),
    "tnet_rbm_trainer_free": (i32, [vp]),
    "tnet_rbm_trainer_add_utterance": (i32, [vp, vp, i32, i32, i32]),
    "tnet_rbm_trainer_finish": (i32, [vp]),
    "tnet_rbm_trainer_steps": (i64, [vp]),
    "tnet_rbm_trainer_stats": (i32, [vp, dp, C.POINTER(i64)]),
    "tnet_rbm_trainer_report": (i32, [vp, C.c_char_p, i32]),
    "tnet_rbm_trainer_prefill": (i64, [vp, vp, i32, i32, i32]),
    "tnet_rbm_trainer_replay": (i32, [vp, i64]),
    "tnet_net_recurrent_get": (i32, [vp, i32, vp, vp]),
    "tnet_net_recurrent_set": (i32, [vp, i32, vp, vp]),
    "tnet_rnn_trainer_create": (vp, [vp, vp, i32, i32]),
    "tnet_rnn_trainer_free": (i32, [vp]),
    "tnet_rnn_trainer_utterance": (i32, [vp, vp, i32, i32, i32, vp]),
    "tnet_rnn_trainer_frames": (i64, [vp]),
    "tnet_gemv_workspace": (i64, [i32, i32]),
    "tnet_gemv_rowvec": (i32, [vp, i32, vp, i32, vp, vp, i32, i32, vp, vp]),
    "tnet_gemv_rows": (i32, [vp, i32, i32, i32, i32, vp, vp, f32, vp, vp]),
    "tnet_rnn_update": (i32, [vp, i32, i32, i32, vp, i32, i32, i32, vp, i32, i32, vp, vp, f32, f32, f32, vp]),
    "tnet_affine_fwd_t": (i32, [vp, MatrixDim, vp, MatrixDim, vp, vp, MatrixDim, i32, vp]),
    "tnet_rbm_update": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, vp]),
    "tnet_rbm_update_stats": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, i32, vp, vp,
                                    vp, vp, vp, vp]),
    "tnet_rbm_update_stats_gather": (i32, [vp, MatrixDim, vp, MatrixDim, vp, MatrixDim, vp, i32, f32, f32, f32, i32, vp,
                                           vp, vp, vp, vp, vp, vp, vp, vp, vp, MatrixDim, MatrixDim, vp]),
    "tnet_rbm_bias_update": (i32, [vp, MatrixDim, i32, vp, vp, f32, f32, vp, vp]),
    "tnet_rbm_stats_update": (i32, [vp, MatrixDim, vp, MatrixDim, i32, vp, vp, vp, vp, f32, f32, vp, vp]),
    "tnet_gemv_rowvec_partial": (i32, [vp, i32, vp, i32, vp, vp, i32, i32, vp, vp]),
    "tnet_rnn_out_partial": (i32, [vp, i32, vp, vp, i32, vp, i32, i32, vp, vp]),
    "tnet_rnn_out_stats": (i32, [vp, i32, i32, vp, vp, vp, vp]),
    "tnet_rnn_out_bwd_update": (i32, [vp, vp, i32, i32, vp, vp, i32, vp, i32, vp, i32, vp, vp, f32, f32, f32, vp, vp,
                                      vp, vp, vp, vp, i32, vp]),
    "tnet_rnn_out_full": (i32, [vp, i32, vp, vp, i32, vp, i32, i32, vp, vp, vp, vp]),
    "tnet_gemv_rowvec_partial_update": (i32, [vp, i32, vp, i32, vp, vp, i32, i32, vp, vp, i32, i32, i32, vp, i32, i32,
                                              vp, vp, f32, f32, f32, vp]),
    "tnet_argmax_correct": (i32, [vp, vp, i32, i32, vp, vp]),
    "tnet_rnn_out_full_ahead": (i32, [vp, i32, vp, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp, i32, i32, f32, f32, f32,
                                      vp, vp, vp, vp, i32, i32, vp, i32, i32, i32, vp]),
    "tnet_rnn_out_bwd_update_ahead": (i32, [vp, vp, i32, i32, vp, vp, i32, vp, i32, vp, i32, vp, vp, f32, f32, f32, vp,
                                            vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, i32,
                                            i32, i32, i32, vp]),
    "tnetF_rand": (i32, [vp, MatrixDim, vp, vp, vp, vp, vp]),
    "tnetF_gauss_rand": (i32, [vp, MatrixDim, vp, vp, vp, vp, vp]),
    "tnetF_binarize_probs": (i32, [vp, vp, vp, MatrixDim, vp]),
    "tnet_rand_binarize": (i32, [vp, i32, vp, MatrixDim, vp, vp, vp, vp, vp]),
    "tnet_add_gauss_noise": (i32, [vp, MatrixDim, f32, vp, vp, vp, vp, vp]),
    "tnet_dp_plan_round": (i32, [vp, i64, i32, C.POINTER(i64), C.POINTER(i32), i64, C.POINTER(i32)]),
    "tnet_dp_shard_ranges": (i32, [i64, i32, i32, C.POINTER(i64), C.POINTER(i64), C.POINTER(i32)]),
    "tnet_net_set_comm": (i32, [vp, vp]),
    "tnet_comm_set_step_rows": (i32, [vp, i64]),
    "tnet_net_train_empty": (i32, [vp, vp, i64]),
    "tnet_trainer_empty_steps": (i64, [vp]),
}

# int fn(void* user, void* buf, long n, int is_double) -- tnet_host_allreduce_fn
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_int)


def header_symbols():
    """Every function declared in include/tnet_kernels.h and include/tnet_train.h."""
    names = []
    for h in ("tnet_kernels.h", "tnet_train.h"):
        text = open(os.path.join(INCLUDE_DIR, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        names += re.findall(r"\b(tnet\w*)\s*\(", text)
    return sorted(set(names))


def _torch_rocm_dir():
    """torch's bundled ROCm runtime directory, found WITHOUT importing torch (None if absent)."""
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.origin:
        return None
    d = os.path.join(os.path.dirname(spec.origin), "lib")
    return d if os.path.exists(os.path.join(d, "libamdhip64.so")) else None


def hip_runtimes_mapped():
    """Distinct libamdhip64 files mapped into this process (/proc/self/maps)."""
    seen = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if line.strip() else ""
                if "libamdhip64.so" in os.path.basename(p):
                    seen.add(os.path.realpath(p))
    except OSError:
        pass
    return sorted(seen)


def _one_hip_runtime():
    """Exactly one HIP runtime and one RCCL per process, whatever the import order.

    PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 / librccl (torch/lib, RPATH $ORIGIN,
    NEEDED by file name "libamdhip64.so", "librccl.so"); this library links /opt/rocm's by soname
    (libamdhip64.so.7, librccl.so.1).  Loaded before torch, ours makes torch map a second HIP runtime
    and a second RCCL beside it, and any librccl mapped before libtorch_hip -- torch's own copy
    included -- ends the process in "double free or corruption" at exit (reproduced here without a
    GPU).  Loaded after torch, our sonames resolve to torch's already-mapped files: one runtime, one
    RCCL, clean exit.  So when torch is installed it is imported first (bench.py and the DP tests use
    torch.distributed for rendezvous anyway).  TNET_HIP_RUNTIME=system skips this (then the process
    must not import torch later); processes without torch -- the drop-in drivers, C callers -- use
    /opt/rocm's runtime."""
    if os.environ.get("TNET_HIP_RUNTIME", "") == "system" or _torch_rocm_dir() is None:
        return
    import torch  # noqa: F401


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise TnetError(f"{LIB_PATH} not built: run `make -C nnet-asr_amd` (or __graft_entry__.build())")
        _one_hip_runtime()
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        rt = hip_runtimes_mapped()
        if len(rt) > 1:
            raise TnetError("two HIP runtimes mapped into one process: " + ", ".join(rt) +
                            " (load libtnet_amd through tnet_amd, or set TNET_HIP_RUNTIME consistently)")
        # (a diagnostic variant -- e.g. an earlier round's build for a same-box A/B -- may lack newer entry points)
        variant = bool(os.environ.get("TNET_LIB_VARIANT"))
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name, None) if variant else getattr(L, name)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status, what=""):
    if status != 0:
        L = lib()
        msg = L.tnet_last_error().decode(errors="replace") or L.tnet_status_str(status).decode()
        raise TnetError(f"{what}: status {status}: {msg}")
    return status


def check_ptr(p, what=""):
    if not p:
        raise TnetError(f"{what}: {lib().tnet_last_error().decode(errors='replace')}")
    return p
