"""ctypes binding of libdssm.so (include/dssm.h).

torch is imported first on purpose: the torch wheel bundles its own libamdhip64.so.7; loading
it before libdssm.so makes the dynamic loader resolve our NEEDED libamdhip64.so.7 to that same
runtime instance, so torch-allocated device pointers and torch stream handles are valid in our
kernels.  There is no fallback: if the library is missing every device call raises."""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the library load, see module doc)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdssm.so")
# diagnostics only: an alternative in-tree build of the same library (A/B of compile-time variants)
LIB_PATH = os.environ.get("DSSM_LIB_PATH", LIB_PATH)

DSSM_ABI_VERSION = 2
DSSM_MAX_LAYERS = 8
DSSM_F32, DSSM_BF16, DSSM_I32 = 0, 1, 2
DSSM_ACT_NONE, DSSM_ACT_RELU = 0, 1
(BUF_LOSS, BUF_COS_SIM_RAW, BUF_COS_SIM, BUF_PROB, BUF_QUERY_NORM, BUF_EMBED, BUF_Z,
 BUF_BATCH_MEAN, BUF_BATCH_VAR, BUF_DZ) = range(10)
BUF_A, BUF_DA = 11, 12
PROBE_SPMM_FWD, PROBE_DW1, PROBE_ADAM, PROBE_CSC = range(4)
# the phases of a data-parallel step graph's last step (include/dssm.h DSSM_PROBE_DP_*)
DP_PROBES = {"fwd_bwd": 4, "grad_pass": 5, "all_to_all": 6, "tail_allreduce": 7, "all_gather": 8,
             "shadow_rebuild": 9}
GRAPH_FWD_BWD, GRAPH_ADAM, GRAPH_SHADOWS, GRAPH_WIRE_SHADOWS = 1, 2, 4, 8
# dssm_plan_schedule bits (include/dssm.h DSSM_SCHED_*)
SCHED_BITS = {"FUSED_STATS": 1, "MERGED_CSC": 2, "HEAVY_IN_ADAM": 4, "FUSED_W1_ADAM": 8,
              "WHOLEK": 16, "DW_IN_APPLY": 32, "SCATTER_IN_COS": 64, "DETERMINISTIC": 128, "NT32": 256,
              "BNB_IN_PAIR": 512, "FWD32": 1024}
# dssm_plan_set_option ids (include/dssm.h DSSM_OPT_*)
OPTIONS = {k: i for i, k in enumerate(["FUSED_STATS", "MERGED_CSC", "HEAVY_IN_ADAM", "SCATTER_IN_COS",
                                         "DW_IN_APPLY", "WIRE_GRAD_PASS", "CSC_RANK", "DETERMINISTIC",
                                         "FUSED_W1_ADAM", "RANK_IN_ADAM", "MEMCPY_NODES", "BNB_IN_PAIR",
                                         "TAIL_IN_A2A", "FWD32"])}


class DssmError(RuntimeError):
    pass


class dssm_shadow_seg(C.Structure):
    """include/dssm.h dssm_shadow_seg: a [rows x cols] weight block at p + offset and its bf16 shadow."""
    _fields_ = [("offset", C.c_int64), ("rows", C.c_int64), ("cols", C.c_int), ("ld", C.c_int), ("ptr", C.c_void_p)]


class dssm_config(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int), ("trigram_d", C.c_int), ("n_layers", C.c_int),
        ("widths", C.c_int * DSSM_MAX_LAYERS), ("query_bs", C.c_int), ("neg", C.c_int),
        ("max_nnz", C.c_int), ("compute_dtype", C.c_int), ("gamma", C.c_float),
        ("bn_eps", C.c_float), ("ema_decay", C.c_float), ("lr", C.c_float), ("beta1", C.c_float),
        ("beta2", C.c_float), ("adam_eps", C.c_float),
    ]


class dssm_segment(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("offset", C.c_int64), ("rows", C.c_int64),
                ("cols", C.c_int64)]


_P = C.c_void_p
_SIGS = {
    "dssm_abi_version": (C.c_int, []),
    "dssm_last_error": (C.c_char_p, []),
    "dssm_config_check": (C.c_int, [C.POINTER(dssm_config)]),
    "dssm_param_count": (C.c_int64, [C.POINTER(dssm_config)]),
    "dssm_param_layout": (C.c_int, [C.POINTER(dssm_config), C.POINTER(dssm_segment), C.c_int]),
    "dssm_ema_count": (C.c_int64, [C.POINTER(dssm_config)]),
    "dssm_workspace_bytes": (C.c_size_t, [C.POINTER(dssm_config)]),
    "dssm_plan_create": (C.c_int, [C.POINTER(dssm_config), _P, C.c_size_t, _P, _P, _P, _P, _P,
                                   C.POINTER(_P)]),
    "dssm_plan_destroy": (C.c_int, [_P]),
    "dssm_plan_buffer": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(_P), C.POINTER(C.c_size_t)]),
    "dssm_plan_set_batch": (C.c_int, [_P, _P, _P, _P]),
    "dssm_plan_sync_shadows": (C.c_int, [_P, _P]),
    "dssm_plan_forward": (C.c_int, [_P, C.c_int, _P]),
    "dssm_plan_backward": (C.c_int, [_P, _P]),
    "dssm_plan_adam": (C.c_int, [_P, C.c_float, _P]),
    "dssm_plan_set_adam_state": (C.c_int, [_P, C.c_float, C.c_float, _P]),
    "dssm_plan_get_adam_state": (C.c_int, [_P, C.POINTER(C.c_float), C.POINTER(C.c_float), _P]),
    "dssm_plan_train_step": (C.c_int, [_P, _P]),
    "dssm_plan_graph_build": (C.c_int, [_P, C.c_int, C.c_float, C.c_int, _P, C.POINTER(C.c_int)]),
    "dssm_plan_graph_launch": (C.c_int, [_P, C.c_int, _P]),
    "dssm_plan_graph_build_steps": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.c_int,
                                              C.c_int, _P, C.POINTER(C.c_int)]),
    "dssm_plan_set_option": (C.c_int, [_P, C.c_int, C.c_int]),
    "dssm_plan_get_option": (C.c_int, [_P, C.c_int]),
    "dssm_plan_fused_stats": (C.c_int, [_P]),
    "dssm_plan_schedule": (C.c_int, [_P]),
    "dssm_plan_set_adam_range": (C.c_int, [_P, C.c_int64, C.c_int64]),
    "dssm_plan_finalize_loss": (C.c_int, [_P, _P]),
    "dssm_plan_graph_probe_read": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(C.c_float)]),
    "dssm_plan_graph_topology": (C.c_int, [_P, C.c_int, C.POINTER(C.c_int64)]),
    "dssm_plan_set_fused_w1_adam": (C.c_int, [_P, C.c_int]),
    "dssm_plan_wire_extent": (C.c_int64, [_P]),
    "dssm_plan_dp_wire_size": (C.c_int64, [_P, C.c_int, C.c_int]),
    "dssm_plan_set_dp_wire": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P, _P, _P, C.c_int64]),
    "dssm_plan_dp_geometry": (C.c_int, [_P, C.POINTER(C.c_int64)]),
    "dssm_plan_wire_shadows": (C.c_int, [_P, _P]),
    "dssm_plan_graph_build_dp_steps": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.c_int,
                                                 C.c_float, C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, _P,
                                                 C.POINTER(C.c_int)]),
    "dssm_plan_probe_enable": (C.c_int, [_P, C.c_int, C.c_int]),
    "dssm_plan_probe_read": (C.c_int, [_P, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int)]),
    "dssm_spmm_csr_fwd": (C.c_int, [_P, _P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, _P, _P,
                                    C.c_int, _P]),
    "dssm_dense_fwd": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P,
                                 _P, C.c_int, _P]),
    "dssm_spmm_csr_fwd_act": (C.c_int, [_P, _P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, _P, _P,
                                        C.c_int, C.c_int, _P]),
    "dssm_dense_fwd_act": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P,
                                     _P, C.c_int, C.c_int, _P]),
    "dssm_spmm_csr_fwd_ex": (C.c_int, [_P, _P, _P, C.c_int, _P, C.c_int, C.c_int, C.c_int, _P, _P, C.c_int,
                                       C.c_int, C.c_int, _P]),
    "dssm_bn_ws_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "dssm_bn_relu_fwd": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_float,
                                   C.c_float, C.c_int, C.c_int, _P, C.c_int, _P, _P, _P, _P]),
    "dssm_cosine_softmax_loss": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, _P,
                                           _P, _P, _P, _P, _P, _P, _P]),
    "dssm_cosine_softmax_loss_dropout": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                                   C.c_uint32, C.c_uint32, C.c_float, _P, _P, _P, _P, _P, _P,
                                                   _P, _P, _P]),
    "dssm_text_clean": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "dssm_vocab_create": (C.c_int, [C.POINTER(_P)]),
    "dssm_vocab_destroy": (C.c_int, [_P]),
    "dssm_vocab_fit": (C.c_int, [_P, C.POINTER(C.c_char_p), C.c_int64]),
    "dssm_vocab_finalize": (C.c_int64, [_P]),
    "dssm_vocab_size": (C.c_int64, [_P]),
    "dssm_vocab_name": (C.c_int, [_P, C.c_int64, C.c_char_p, C.c_size_t]),
    "dssm_vocab_add": (C.c_int, [_P, C.c_char_p]),
    "dssm_crc32c": (C.c_uint32, [C.c_uint32, _P, C.c_size_t]),
    "dssm_vocab_transform": (C.c_int, [_P, C.POINTER(C.c_char_p), C.c_int64, _P, _P, _P, C.c_int64,
                                       C.POINTER(C.c_int64)]),
    "dssm_feeder_create": (C.c_int, [C.POINTER(_P), C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_int64),
                                     C.c_int, C.c_int, C.c_int64, C.c_int, C.POINTER(_P)]),
    "dssm_feeder_submit": (C.c_int, [_P, C.c_int, C.c_int64]),
    "dssm_feeder_acquire": (C.c_int, [_P, C.c_int, _P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P),
                                      C.POINTER(C.c_int64)]),
    "dssm_feeder_release": (C.c_int, [_P, C.c_int, _P]),
    "dssm_feeder_destroy": (C.c_int, [_P]),
    "dssm_rnn_ws_floats": (C.c_size_t, [C.c_int, C.c_int, C.c_int, C.c_int]),
    "dssm_rnn_forward": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.POINTER(_P), _P, _P,
                                   C.c_int, _P]),
    "dssm_rnn_dropout": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_float, C.c_uint32, C.c_uint32,
                                   C.c_float, _P]),
    "dssm_rnn_backward": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_P), _P, C.c_int,
                                    _P, _P, C.c_int64, C.POINTER(_P), _P]),
    "dssm_rnn_adam": (C.c_int, [_P, _P, _P, _P, C.c_int64, C.c_int64, _P, C.c_float, C.c_float, C.c_float,
                                C.c_float, _P]),
    "dssm_rnn_adam_ex": (C.c_int, [_P, _P, _P, _P, C.c_int64, C.c_int64, _P, C.c_float, C.c_float, C.c_float,
                                   C.c_float, _P, _P]),
    "dssm_rnn_bf16_emb16_offset": (C.c_size_t, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "dssm_rnn_bf16_forward_ex": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.POINTER(_P), _P,
                                           _P, C.c_int, C.c_int, _P]),
    "dssm_rnn_bf16_supported": (C.c_int, [C.c_int, C.c_int]),
    "dssm_rnn_bf16_ws_bytes": (C.c_size_t, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "dssm_rnn_bf16_forward": (C.c_int, [_P, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.POINTER(_P),
                                        _P, _P, C.c_int, _P]),
    "dssm_rnn_bf16_backward": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_P), _P,
                                         C.c_int, _P, _P, C.POINTER(_P), _P]),
    "dssm_rnn_bf16_probe": (C.c_int, [C.c_int]),
    "dssm_rnn_bf16_probe_read": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "dssm_spmm_bwd_ws_bytes": (C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    "dssm_spmm_csr_bwd_w": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int,
                                      _P, _P, _P]),
    "dssm_cosine_softmax_loss_mapped": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_float, _P, _P,
                                                  _P, _P, _P, _P, _P, _P]),
    "dssm_csc_transpose": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, _P, _P]),
    "dssm_adam_probe": (C.c_int, [C.c_int]),
    "dssm_adam_probe_read": (C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "dssm_rows_gather_sum": (C.c_int, [_P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_float, _P, C.c_int, _P,
                                       C.c_int, _P]),
    "dssm_rows_gather_sum_ex": (C.c_int, [_P, C.c_int, _P, _P, C.c_int, C.c_int, C.c_float, _P, C.c_int, _P,
                                          C.c_int, C.c_int, _P]),
    "dssm_dense_bwd_slab_floats": (C.c_size_t, [C.c_int, C.c_int, C.c_int, C.c_int]),
    "dssm_dense_bwd": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P, C.c_int,
                                 _P, C.c_int, _P, _P, _P]),
    "dssm_dense_bwd_masked": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P,
                                        C.c_int, _P, C.c_int, _P, C.c_int, _P, _P, _P]),
    "dssm_dense_bwd_ex": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _P, C.c_int,
                                    _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, _P, _P, _P, _P]),
    "dssm_bn_relu_bwd": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P, _P, _P, _P, C.c_float, C.c_int, _P,
                                   C.c_int, _P, C.c_int, _P, _P, _P]),
    "dssm_adam_step": (C.c_int, [_P, _P, _P, _P, C.c_int64, C.c_float, C.c_float, C.c_float, C.c_float, _P,
                                 C.c_float, C.c_int, _P]),
    "dssm_adam_step_shadow": (C.c_int, [_P, _P, _P, _P, _P, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float,
                                        _P, C.c_float, C.c_int, _P, C.c_int, _P]),
    "dssm_spmm_bwd_w_adam": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int,
                                       _P, _P, _P, _P, C.c_int64, C.c_int64, _P, C.c_int64, C.c_int, _P, C.c_int,
                                       _P, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, _P, C.c_float,
                                       C.c_int, C.c_int, _P, C.c_int, _P, _P]),
    "dssm_spmm_bwd_csc": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, C.c_int, _P, _P]),
    "dssm_adam_tickets_bytes": (C.c_size_t, [C.c_int]),
    "dssm_adam_probe_span": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "dssm_adam_advance": (C.c_int, [_P, C.c_float, C.c_float, _P]),
    "dssm_rows_gather": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, _P, C.c_int, _P]),
    "dssm_rows_scatter_add": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, _P]),
    "dssm_relu": (C.c_int, [_P, C.c_int, C.c_int, C.c_int, _P, C.c_int, _P]),
    "dssm_relu_bwd": (C.c_int, [_P, C.c_int, _P, C.c_int, C.c_int, C.c_int, _P, C.c_int, _P]),
    "dssm_comm_unique_id": (C.c_int, [_P]),
    "dssm_comm_init": (C.c_int, [C.c_int, C.c_int, _P]),
    "dssm_allreduce_sum_f32": (C.c_int, [_P, C.c_int64, _P]),
    "dssm_comm_world": (C.c_int, []),
    "dssm_comm_info": (C.c_int, [_P, _P, _P]),
    "dssm_allreduce_sum": (C.c_int, [_P, C.c_int64, C.c_int, _P]),
    "dssm_reduce_scatter_sum": (C.c_int, [_P, _P, C.c_int64, C.c_int, _P]),
    "dssm_all_gather": (C.c_int, [_P, _P, C.c_int64, C.c_int, _P]),
    "dssm_all_to_all": (C.c_int, [_P, _P, C.c_int64, C.c_int, _P]),
    "dssm_all_to_allv": (C.c_int, [_P, _P, _P, _P, C.c_int, _P, C.c_int64, C.c_int, _P]),
    "dssm_all_to_all_tail": (C.c_int, [_P, _P, C.c_int64, C.c_int, _P, C.c_int64, _P]),
    "dssm_rows_pack_u16": (C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, _P]),
    "dssm_rows_unpack_u16": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_int64, C.c_int64, _P, _P]),
    "dssm_comm_destroy": (C.c_int, []),
    # peer-store exchange (csrc/peer.hip)
    "dssm_peer_alloc": (C.c_int, [C.c_int64, _P]),
    "dssm_peer_free": (C.c_int, [_P]),
    "dssm_peer_can_access": (C.c_int, [C.c_int, _P]),
    "dssm_ipc_handle": (C.c_int, [_P, _P]),
    "dssm_ipc_open": (C.c_int, [_P, _P]),
    "dssm_ipc_close": (C.c_int, [_P]),
    "dssm_plan_set_dp_peers": (C.c_int, [_P, C.c_int, _P, _P, _P, _P]),
    "dssm_plan_set_peer_timeout": (C.c_int, [_P, C.c_double]),
    "dssm_plan_peer_exchange": (C.c_int, [_P, C.c_int, _P]),
    "dssm_plan_peer_status": (C.c_int, [_P, _P]),
    "dssm_plan_peer_selftest": (C.c_int, [_P, _P, _P]),
}
PEER_FLAG_BYTES = 4096  # include/dssm.h DSSM_PEER_FLAG_BYTES

_lib = None


def load(path: str = LIB_PATH):
    """Load libdssm.so (once).  Raises DssmError when it is missing — no CPU fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DssmError(f"{path} not found: build it with `python -m dssm_amd.build` "
                        "(the HIP path has no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.dssm_abi_version() != DSSM_ABI_VERSION:
        raise DssmError("libdssm.so ABI version mismatch")
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS)


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().dssm_last_error().decode(errors="replace")
        raise DssmError(f"{what or 'dssm call'} failed ({rc}): {msg}")


def ptr(t) -> int:
    """Device pointer of a torch tensor (0 for None)."""
    return 0 if t is None else t.data_ptr()


def stream_ptr(stream=None) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream
