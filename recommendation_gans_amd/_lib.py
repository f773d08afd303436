"""ctypes binding of librg_hip.so (include/rg_hip.h).

There is deliberately no CPU fallback: if the library is missing or cannot be
loaded, every entry point raises ``RuntimeError``.  ``torch`` is imported
before the library so that the HIP runtime torch ships (SONAME
libamdhip64.so.7) is the one librg_hip.so binds to.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede loading the HIP library)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "librg_hip.so")

RG_OK = 0
RG_MF_LIST_CAP = 8
RG_MF_MAX_NEG = 8
RG_COMM_ID_BYTES = 128
RG_MT_PAD = 1280

LOSS_KINDS = {"pointwise": 0, "bpr": 1, "hinge": 2, "adaptive_hinge": 3,
              "pointwise_pos": 4}   # implicit.py:359-360 (neg_examples=None): BCE on the positives only
OPT_KINDS = {"adam": 0, "sgd": 1, "rms": 2}

c_f32p = ctypes.POINTER(ctypes.c_float)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
# rg_host_allreduce_fn (include/rg_hip.h): int (*)(void *ctx, float *host_buf, int64_t n)
HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
# rg_host_gather_fn: int (*)(void *ctx, const uint32_t *send, int64_t n, uint32_t *recv)
HOST_GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)


class MFTables(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "user_w", "item_w", "user_b", "item_b",
        "user_w_out", "item_w_out", "user_b_out", "item_b_out",
        "user_w_m", "user_w_v", "item_w_m", "item_w_v",
        "user_b_m", "user_b_v", "item_b_m", "item_b_v")] + [
        ("num_users", ctypes.c_int64), ("num_items", ctypes.c_int64),
        ("dim", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class MFBatch(ctypes.Structure):
    _fields_ = [("pos_user", ctypes.c_void_p), ("pos_item", ctypes.c_void_p),
                ("n_pos", ctypes.c_int64), ("cols", ctypes.c_int64), ("col_offset", ctypes.c_int64),
                ("global_cols", ctypes.c_int64), ("global_pos", ctypes.c_int64), ("neg_cols", ctypes.c_int64),
                ("words", ctypes.c_void_p), ("pool", ctypes.c_void_p), ("pool_len", ctypes.c_int64),
                ("n_neg", ctypes.c_int32), ("loss", ctypes.c_int32), ("pairs", ctypes.c_void_p)]


class MFWork(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "row_count", "row_list", "hot_grad", "hot_bias_grad", "loss_partials", "scores",
        "max_key", "active_count", "plan_perm", "plan_pos_slot", "plan_item_slot_off",
        "part_row", "part_bias")] + [("claim_num_users", ctypes.c_int64)]


class MFMark(ctypes.Structure):
    _fields_ = [("stamp", ctypes.c_void_p), ("num_users", ctypes.c_int64), ("serial", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


class MFPipe(ctypes.Structure):
    _fields_ = [("hot_users", ctypes.c_void_p), ("nhot", ctypes.c_void_p), ("counts_next", ctypes.c_void_p),
                ("gate", ctypes.c_void_p), ("gate_next", ctypes.c_void_p), ("nhot_free", ctypes.c_void_p),
                ("hot_out", ctypes.c_void_p), ("nhot_out", ctypes.c_void_p), ("err", ctypes.c_void_p)]


class MFLoss(ctypes.Structure):
    _fields_ = [("n_partials", ctypes.c_int64), ("inv_a", ctypes.c_double), ("inv_b", ctypes.c_double),
                ("out", ctypes.c_void_p)]


class Opt(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("alpha", ctypes.c_float), ("one_minus_beta1", ctypes.c_float),
                ("one_minus_beta2", ctypes.c_float), ("one_minus_alpha", ctypes.c_float),
                ("step_size", ctypes.c_float),
                ("bias_correction2_sqrt", ctypes.c_float)]


class MTGen(ctypes.Structure):
    _fields_ = [("state", ctypes.c_void_p), ("out", ctypes.c_void_p), ("state_before", ctypes.c_void_p),
                ("nwords", ctypes.c_int64)]


class MFStepperConfig(ctypes.Structure):
    _fields_ = [("tables", MFTables * 2), ("work", MFWork), ("mt_state", ctypes.c_void_p),
                ("pairs", ctypes.c_void_p * 2),
                ("pool", ctypes.c_void_p), ("pool_len", ctypes.c_int64), ("n_neg", ctypes.c_int32),
                ("loss", ctypes.c_int32), ("cols", ctypes.c_int64), ("col_offset", ctypes.c_int64),
                ("global_cols", ctypes.c_int64), ("neg_cols", ctypes.c_int64), ("item_grad", ctypes.c_void_p),
                ("comm", ctypes.c_void_p), ("opt", Opt), ("lr_d", ctypes.c_double), ("beta1_d", ctypes.c_double),
                ("beta2_d", ctypes.c_double), ("step", ctypes.c_int64), ("n_partials", ctypes.c_int64),
                ("current_set", ctypes.c_int32), ("gen_mode", ctypes.c_int32),
                ("dp_mode", ctypes.c_int32), ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("pad2_", ctypes.c_int32), ("shard_users", ctypes.c_int64), ("shard_items", ctypes.c_int64),
                ("grad_buf", ctypes.c_void_p), ("owner_rec", ctypes.c_void_p * 2), ("owner_seg", ctypes.c_void_p * 2),
                ("owner_scores", ctypes.c_void_p * 2)]


class NCFModel(ctypes.Structure):
    _fields_ = [("user_w", ctypes.c_void_p), ("item_w", ctypes.c_void_p), ("user_w_m", ctypes.c_void_p),
                ("user_w_v", ctypes.c_void_p), ("item_w_m", ctypes.c_void_p), ("item_w_v", ctypes.c_void_p),
                ("mlp", ctypes.c_void_p), ("mlp_m", ctypes.c_void_p), ("mlp_v", ctypes.c_void_p),
                ("num_users", ctypes.c_int64), ("num_items", ctypes.c_int64), ("dim", ctypes.c_int32),
                ("mf_dim", ctypes.c_int32), ("mf_user_w", ctypes.c_void_p), ("mf_item_w", ctypes.c_void_p),
                ("mf_user_m", ctypes.c_void_p), ("mf_user_v", ctypes.c_void_p), ("mf_item_m", ctypes.c_void_p),
                ("mf_item_v", ctypes.c_void_p)]


class NCFWork(ctypes.Structure):
    _fields_ = [("contrib", ctypes.c_void_p), ("mlp_partials", ctypes.c_void_p), ("scores", ctypes.c_void_p),
                ("dp", ctypes.c_void_p), ("mask_pos", ctypes.c_void_p), ("mask_neg", ctypes.c_void_p),
                ("seed", ctypes.c_uint64), ("training", ctypes.c_int32), ("tile_rows", ctypes.c_int32),
                ("mf_contrib", ctypes.c_void_p), ("mf_hot_grad", ctypes.c_void_p), ("mf_part_row", ctypes.c_void_p)]


class GANDims(ctypes.Structure):
    _fields_ = [("num_items", ctypes.c_int32), ("slate_size", ctypes.c_int32), ("hidden", ctypes.c_int32),
                ("emb_dim", ctypes.c_int32), ("z_dim", ctypes.c_int32), ("batch_max", ctypes.c_int32)]


class GANModel(ctypes.Structure):
    _fields_ = [("dims", GANDims), ("g", ctypes.c_void_p), ("g_m", ctypes.c_void_p), ("g_v", ctypes.c_void_p),
                ("d", ctypes.c_void_p), ("d_m", ctypes.c_void_p), ("d_v", ctypes.c_void_p)]


class GANBatch(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_int32), ("hist_len", ctypes.c_int32), ("hist", ctypes.c_void_p),
                ("slates", ctypes.c_void_p), ("hist_items", ctypes.c_void_p), ("hist_off", ctypes.c_void_p),
                ("hist_rows", ctypes.c_void_p), ("n_hist_items", ctypes.c_int32), ("n_hits", ctypes.c_int32),
                ("hit_col", ctypes.c_void_p), ("hit_row", ctypes.c_void_p), ("hit_tile_off", ctypes.c_void_p)]


class GANNoise(ctypes.Structure):
    _fields_ = [("z", ctypes.c_void_p), ("masks", ctypes.c_void_p * 8), ("seed", ctypes.c_uint64)]


# rg_gan_layout block indices (include/rg_hip.h enum rg_gan_g_block / rg_gan_d_block)
GAN_G_BLOCKS = ["WH", "BH", "EMB", "W1", "B1", "GAMMA1", "BETA1", "W2", "B2", "GAMMA2", "BETA2",
                "RM1", "RV1", "RM2", "RV2"]
GAN_D_BLOCKS = ["W1S", "EMB", "W1E", "B1", "W2", "B2", "W3", "B3", "W4", "B4"]
GAN_WS_FAKE, GAN_WS_DOUT = 0, 1


class MFLazy(ctypes.Structure):
    _fields_ = [("last_rel", ctypes.c_void_p), ("umark", ctypes.c_void_p), ("step_consts", ctypes.c_void_p),
                ("n_consts", ctypes.c_int64), ("base", ctypes.c_int64), ("step", ctypes.c_int64),
                ("full", ctypes.c_int32), ("pad_", ctypes.c_int32), ("rows_done", ctypes.c_void_p)]


class MFStepIn(ctypes.Structure):
    _fields_ = [("pos_user", ctypes.c_void_p), ("pos_item", ctypes.c_void_p), ("n_pos", ctypes.c_int64),
                ("global_pos", ctypes.c_int64), ("plan_perm", ctypes.c_void_p), ("plan_pos_slot", ctypes.c_void_p),
                ("plan_item_slot_off", ctypes.c_void_p), ("n_planned", ctypes.c_int64)]


class MFOwnerBatch(ctypes.Structure):
    _fields_ = [("pos_user", ctypes.c_void_p), ("pos_item", ctypes.c_void_p), ("n_pos", ctypes.c_int64),
                ("global_cols", ctypes.c_int64), ("plan_perm", ctypes.c_void_p), ("plan_pos_slot", ctypes.c_void_p),
                ("n_planned", ctypes.c_int64), ("words", ctypes.c_void_p), ("pool", ctypes.c_void_p),
                ("pool_len", ctypes.c_int64), ("n_neg", ctypes.c_int32), ("loss", ctypes.c_int32),
                ("world", ctypes.c_int32), ("rank", ctypes.c_int32), ("neg_rec", ctypes.c_void_p),
                ("seg_count", ctypes.c_void_p), ("scores", ctypes.c_void_p), ("claim_count", ctypes.c_void_p),
                ("claim_num_users", ctypes.c_int64)]


# (name, restype, argtypes) for every symbol declared in include/rg_hip.h
SIGNATURES = [
    ("rg_gan_layout", ctypes.c_int, [ctypes.POINTER(GANDims), ctypes.POINTER(ctypes.c_int64),
                                     ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    ("rg_gan_workspace_bytes", ctypes.c_int64, [ctypes.POINTER(GANDims)]),
    ("rg_gan_workspace_offset", ctypes.c_int64, [ctypes.POINTER(GANDims), ctypes.c_int32]),
    ("rg_gan_d_step", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GANModel), ctypes.c_void_p,
                                     ctypes.POINTER(GANBatch), ctypes.POINTER(GANNoise), ctypes.POINTER(Opt),
                                     ctypes.c_void_p]),
    ("rg_gan_g_step", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GANModel), ctypes.c_void_p,
                                     ctypes.POINTER(GANBatch), ctypes.POINTER(GANNoise), ctypes.POINTER(Opt),
                                     ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_gan_generate", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(GANModel), ctypes.c_void_p,
                                       ctypes.POINTER(GANBatch), ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_gemm_ws_mode", ctypes.c_int, [ctypes.c_int32]),
    ("rg_gemm_f32_rms", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_float, ctypes.c_float, ctypes.c_float]),
    ("rg_gemm_f32", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_void_p]),
    ("rg_ncf_mlp_len", ctypes.c_int64, [ctypes.c_int32]),
    ("rg_neumf_param_len", ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    ("rg_ncf_mask_units", ctypes.c_int64, [ctypes.c_int32]),
    ("rg_ncf_cols_per_tile", ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rg_ncf_rows_per_tile", ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    ("rg_ncf_tiles", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rg_ncf_blocks", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rg_ncf_pairs", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(MFBatch),
                                    ctypes.POINTER(MFWork), ctypes.POINTER(NCFWork), ctypes.c_int32]),
    ("rg_ncf_adapt_local", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                          ctypes.POINTER(NCFWork), ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_void_p]),
    ("rg_ncf_adapt_global", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(NCFWork),
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_ncf_adapt_winner", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(NCFWork),
                                           ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    ("rg_ncf_adapt_dp", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(NCFWork),
                                       ctypes.c_void_p]),
    ("rg_ncf_update", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(NCFWork),
                                     ctypes.c_int64, ctypes.POINTER(Opt), ctypes.c_void_p, ctypes.POINTER(MFLoss)]),
    ("rg_ncf_mlp_grad", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(NCFWork),
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(MFLoss), ctypes.c_void_p]),
    ("rg_ncf_mlp_apply", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.c_void_p,
                                        ctypes.POINTER(Opt), ctypes.c_void_p]),
    ("rg_ncf_grads", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(MFWork),
                                    ctypes.POINTER(NCFWork), ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int32]),
    ("rg_ncf_apply_dense", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.c_void_p,
                                          ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]),
    ("rg_ncf_apply", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(MFWork),
                                    ctypes.c_void_p, ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64]),
    ("rg_ncf_tail", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(MFWork),
                                   ctypes.POINTER(NCFWork), ctypes.c_int64, ctypes.POINTER(Opt), ctypes.c_void_p,
                                   ctypes.POINTER(MFLoss), ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                   ctypes.POINTER(MTGen)]),
    ("rg_ncf_tail_validate", ctypes.c_int, [ctypes.POINTER(NCFModel), ctypes.POINTER(MFWork), ctypes.POINTER(NCFWork),
                                            ctypes.c_int64, ctypes.POINTER(Opt), ctypes.c_void_p,
                                            ctypes.POINTER(MFLoss)]),
    ("rg_neumf_apply", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(NCFModel), ctypes.POINTER(MFWork),
                                      ctypes.POINTER(NCFWork), ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64]),
    ("rg_pool_build", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    ("rg_mf_stepper_prefetch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn)]),
    ("rg_mf_stepper_prefetch_inline", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn)]),
    ("rg_mf_stepper_prefetch_args", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                                   ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork)]),
    ("rg_mf_stepper_tail_gen", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MTGen)]),
    ("rg_topk_rows", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_void_p]),
    ("rg_mt_window_host", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]),
    ("rg_mt_window_to_cpython", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("rg_mt_advance_host", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    ("rg_uniform_scratch_len", ctypes.c_int64, [ctypes.c_int64]),
    ("rg_stream_copy", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    ("rg_uniform_int64", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    ("rg_comm_unique_id", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    ("rg_comm_create", ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rg_comm_create_local", ctypes.c_void_p, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rg_comm_create_host", ctypes.c_void_p, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                              ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_comm_set_host_gather", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_comm_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("rg_comm_info", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32)]),
    ("rg_comm_allreduce_sum_f32", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]),
    ("rg_mt_generate", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                      ctypes.c_void_p]),
    ("rg_mf_partials_len", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    ("rg_mf_plan_units_per_block", ctypes.c_int64, [ctypes.c_int32]),
    ("rg_mf_plans_scratch_len", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
    ("rg_mf_plans_build", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_pairs_len", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    ("rg_mf_prepare", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork)]),
    ("rg_mf_prepare_marked", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                            ctypes.POINTER(MFMark)]),
    ("rg_mf_pairs", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFBatch),
                                   ctypes.POINTER(MFWork), ctypes.c_int32]),
    ("rg_mf_apply", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                   ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(MFLoss)]),
    ("rg_mf_apply_prepare", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                           ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(MFLoss),
                                           ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork)]),
    ("rg_mf_apply_prepare_gen", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                               ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64,
                                               ctypes.POINTER(MFLoss), ctypes.POINTER(MFBatch),
                                               ctypes.POINTER(MFWork), ctypes.POINTER(MTGen)]),
    ("rg_mf_prepare_hot", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                         ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_pipe2_hot", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                       ctypes.POINTER(Opt), ctypes.POINTER(MFLoss), ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int64, ctypes.c_void_p, ctypes.POINTER(MTGen)]),
    ("rg_mf_pipe2_cold", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                        ctypes.POINTER(Opt), ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                        ctypes.c_void_p, ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MTGen)]),
    ("rg_mf_pipe_step", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                       ctypes.POINTER(Opt), ctypes.POINTER(MFLoss), ctypes.POINTER(MFBatch),
                                       ctypes.POINTER(MFWork), ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                       ctypes.POINTER(MFPipe), ctypes.POINTER(MTGen)]),
    ("rg_mf_step_front", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFBatch),
                                        ctypes.POINTER(MFWork), ctypes.POINTER(MFMark), ctypes.POINTER(Opt),
                                        ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(MFBatch),
                                        ctypes.POINTER(MFWork), ctypes.POINTER(MFMark)]),
    ("rg_mf_step_cold", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFMark),
                                       ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64]),
    ("rg_mf_step_hot", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFBatch),
                                      ctypes.POINTER(MFWork), ctypes.POINTER(MFMark), ctypes.POINTER(Opt),
                                      ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(MFLoss)]),
    ("rg_mf_grads", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(MFLoss)]),
    ("rg_mf_grad_chunk", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]),
    ("rg_mf_grads_sharded", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                           ctypes.POINTER(MFLoss)]),
    ("rg_mf_apply_shard", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.c_void_p,
                                         ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_void_p]),
    ("rg_mf_item_grad_chunk", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    ("rg_mf_grads_item_shard", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                              ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(MFLoss)]),
    ("rg_mf_apply_item_shard", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.c_void_p,
                                              ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                              ctypes.c_void_p]),
    ("rg_mf_stepper_dp_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                              ctypes.POINTER(MFStepIn), ctypes.c_void_p]),
    ("rg_mf_stepper_dp_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_owner_segments", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    ("rg_mf_owner_rec_len", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32]),
    ("rg_mf_owner_partials_len", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    ("rg_mf_owner_partials_used", ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                   ctypes.c_int64]),
    ("rg_mf_owner_prepare", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFOwnerBatch)]),
    ("rg_mf_owner_adapt", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFOwnerBatch)]),
    ("rg_mf_owner_scores", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFOwnerBatch)]),
    ("rg_mf_owner_back", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFOwnerBatch),
                                        ctypes.POINTER(MFWork)]),
    ("rg_mf_stepper_owner_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn)]),
    ("rg_mf_stepper_owner_mid", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_owner_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_owner_scores", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_owner_loss", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFOwnerBatch), ctypes.c_void_p]),
    ("rg_mf_stepper_owner_val_end", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_owner_val", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                               ctypes.c_void_p]),
    ("rg_comm_reduce_scatter_f32", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_int64]),
    ("rg_comm_allgather_f32", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    ("rg_mf_apply_dense", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.c_void_p,
                                         ctypes.POINTER(Opt), ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]),
    ("rg_loss_finalize", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double,
                                        ctypes.c_double, ctypes.c_void_p]),
    ("rg_mf_scores", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int64, ctypes.c_void_p]),
    ("rg_mf_stepper_mt_mode", ctypes.c_int32, [ctypes.c_void_p]),
    ("rg_mf_stepper_create", ctypes.c_void_p, [ctypes.POINTER(MFStepperConfig)]),
    ("rg_mf_stepper_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("rg_mf_stepper_train", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                           ctypes.POINTER(MFStepIn), ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p]),
    ("rg_mf_stepper_train_ahead", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                                 ctypes.POINTER(MFStepIn), ctypes.POINTER(MFStepIn), ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_pipe_error", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_pipelined", ctypes.c_int, [ctypes.c_void_p]),
    ("rg_mf_stepper_acquire", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(MFStepIn),
                                             ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork)]),
    ("rg_mf_stepper_release", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_opt", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(Opt)]),
    ("rg_mf_stepper_state", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_advance", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64]),
    ("rg_mf_stepper_sync_mt", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]),
    ("rg_mf_stepper_flush", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_mf_stepper_lazy_count", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("rg_mf_pairs_prepare", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFBatch),
                                           ctypes.POINTER(MFWork), ctypes.POINTER(MFBatch), ctypes.POINTER(MFWork),
                                           ctypes.c_void_p, ctypes.c_int32]),
    ("rg_mf_apply_lazy", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(MFWork),
                                        ctypes.POINTER(Opt), ctypes.POINTER(MFLoss), ctypes.POINTER(MFLazy),
                                        ctypes.POINTER(MTGen)]),
    ("rg_mf_lazy_flush", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MFTables), ctypes.POINTER(Opt),
                                        ctypes.POINTER(MFLazy)]),
    ("rg_event_elapsed_ms", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("rg_last_error", ctypes.c_char_p, []),
    ("rg_version", ctypes.c_char_p, []),
    ("rg_build_flags", ctypes.c_int32, []),
]

_lib = None
_load_error = None


def load(path=None):
    """Load librg_hip.so (once) and bind every exported entry point."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    p = path or os.environ.get("RG_LIB") or LIB_PATH      # RG_LIB: a same-box A/B variant (scripts)
    if not os.path.exists(p):
        raise RuntimeError(f"librg_hip.so not found at {p}: build it with "
                           "`python -m recommendation_gans_amd.build` (hipcc, gfx950). "
                           "There is no CPU fallback for the hot path.")
    try:
        L = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover
        _load_error = e
        raise RuntimeError(f"cannot load {p}: {e}") from e
    for name, res, args in SIGNATURES:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


RG_BUILD_AB = 1


def ab_build():
    """True when the loaded library is an A/B build (RG_AB): only then do the measured-slower
    alternatives' RG_* switches select anything."""
    return bool(load().rg_build_flags() & RG_BUILD_AB)


def check(rc, what):
    if rc != RG_OK:
        msg = load().rg_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def elapsed_ms(ev_begin, ev_end):
    """Elapsed time of a torch.cuda.Event pair recorded natively (rg_mf_stepper_train)."""
    ms = ctypes.c_float()
    check(load().rg_event_elapsed_ms(ctypes.c_void_p(ev_begin.cuda_event), ctypes.c_void_p(ev_end.cuda_event),
                                     ctypes.byref(ms)), "rg_event_elapsed_ms")
    return ms.value


def require_gpu(tensor_or_device=None):
    if not torch.cuda.is_available():
        raise RuntimeError("the recommendation_gans_amd hot path runs on an MI355X (ROCm) GPU only; "
                           "torch.cuda.is_available() is False")
