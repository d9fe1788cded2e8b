"""ctypes binding of libavt.so (the C-ABI declared in include/avt.h) and its build recipe.

The library is built in-tree (``audio-visual-tubes_amd/libavt.so``) with
``hipcc --offload-arch=gfx950``; it travels to the GPU box with the repo snapshot.  There is no
CPU fallback: every op raises if the library or a GPU is missing.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libavt.so")
# A/B measurement only: load another in-tree build of the same ABI (e.g. libavt_base.so)
LOAD_PATH = os.environ.get("AVT_LIB_PATH", LIB_PATH)
SOURCES = ["conv_gemm.hip", "bn.hip", "pool.hip", "head.hip", "misc.hip", "tube.hip", "eval.hip", "audio.hip", "frames.hip"]

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_F = ctypes.c_float
_Z = ctypes.c_size_t

class DgradBnEpi(ctypes.Structure):
    """avt_dgrad_bn_epi (include/avt.h): the BatchNorm-backward epilogue of avt_conv2d_dgrad_bn."""
    _fields_ = [("xc", ctypes.c_void_p), ("y", ctypes.c_void_p), ("stats", ctypes.c_void_p),
                ("acc", ctypes.c_void_p), ("xc2", ctypes.c_void_p), ("stats2", ctypes.c_void_p),
                ("acc2", ctypes.c_void_p), ("skip_class00", ctypes.c_int), ("append_slots", ctypes.c_int)]


class BnBwdTarget(ctypes.Structure):
    """avt_bn_bwd_target (include/avt.h): one BatchNorm fed by the masked gradient of avt_bn_bwd_mask."""
    _fields_ = [("xc", ctypes.c_void_p), ("mean", ctypes.c_void_p), ("invstd", ctypes.c_void_p),
                ("gamma", ctypes.c_void_p), ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p),
                ("gc", ctypes.c_void_p), ("workspace", ctypes.c_void_p)]


class SlabReduceDesc(ctypes.Structure):
    """avt_slab_reduce_desc (include/avt.h): a wgrad split-K slab left for avt_wgrad_reduce_batch."""
    _fields_ = [("slab", ctypes.c_void_p), ("dw", ctypes.c_void_p), ("splits", ctypes.c_int), ("tiles", ctypes.c_int),
                ("nnt", ctypes.c_int), ("Mg", ctypes.c_int), ("ldw", ctypes.c_int), ("wm", ctypes.c_int),
                ("wn", ctypes.c_int), ("tm", ctypes.c_int), ("tn", ctypes.c_int)]


# name -> (restype, argtypes)
SIGNATURES = {
    "avt_last_error": (ctypes.c_char_p, []),
    "avt_abi_version": (_I, []),
    "avt_build_flags": (_I, []),
    "avt_peak_mfma": (_I, [_P, _I, _I, _I, ctypes.c_uint, _P]),
    "avt_peak_mfma_flops": (_L, [_I, _I, _I]),
    "avt_copy16": (_I, [_P, _P, _Z, _I, _P]),
    "avt_set_conv_variant": (_I, [_I]),
    "avt_set_wgrad_policy": (_I, [_I, _I]),
    "avt_set_nt64_config": (_I, [_I]),
    "avt_set_halo": (_I, [_I]),
    "avt_set_halo8": (_I, [_I]),
    "avt_set_halo8_nst": (_I, [_I]),
    "avt_conv_stem_dgrad": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "avt_set_halo8_form": (_I, [_I]),
    "avt_set_halo_stages": (_I, [_I, _I]),
    "avt_set_c64": (_I, [_I]),
    "avt_set_s2_dgrad_one": (_I, [_I]),
    "avt_set_stem_kernel": (_I, [_I]),
    "avt_set_stem_wgrad": (_I, [_I]),
    "avt_set_nt128_config": (_I, [_I]),
    "avt_set_wgrad_slab_max": (_I, [_I, _I]),
    "avt_set_wgrad_tiles": (_I, [_I]),
    "avt_set_small_tiles": (_I, [_I]),
    "avt_set_wgrad_halo": (_I, [_I]),
    "avt_set_wgrad_row3": (_I, [_I, _I, _I]),
    "avt_set_halo3d": (_I, [_I]),
    "avt_set_halo_tps2": (_I, [_I]),
    "avt_set_wgrad_fused": (_I, [_I, _I]),
    "avt_conv2d_wgrad_tickets": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "avt_conv2d_wgrad_tk": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _Z, _P, _I, _P]),
    "avt_conv2d_wgrad_defer": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _Z,
                                    ctypes.POINTER(SlabReduceDesc), _P]),
    "avt_wgrad_reduce_batch": (_I, [ctypes.POINTER(SlabReduceDesc), _I, _P]),
    "avt_bn_acc_doubles": (_Z, [_L, _I]),
    "avt_conv2d_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "avt_conv2d_dgrad": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "avt_conv2d_dgrad_bn": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, ctypes.POINTER(DgradBnEpi), _P]),
    "avt_bn_bwd_premasked": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P]),
    "avt_conv2d_dgrad_mask": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "avt_conv2d_splitk_plan": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "avt_set_halo_splitk": (_I, [_I, _I]),
    "avt_set_wgrad_nst": (_I, [_I, _I]),
    "avt_set_wgrad_slots_pct": (_I, [_I]),
    "avt_conv2d_fwd_ws": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _L, _P, _I, _P]),
    "avt_conv2d_dgrad_ws": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _L, _P, _I, _P]),
    "avt_bn_apply_mask": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P]),
    "avt_bn_bwd_mask": (_I, [_P, _P, ctypes.POINTER(BnBwdTarget), ctypes.POINTER(BnBwdTarget), _L, _I, _P]),
    "avt_conv2d_wgrad_workspace": (_Z, [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "avt_conv2d_wgrad": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _Z, _P]),
    "avt_bn_finalize": (_I, [_P, _L, _I, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P]),
    "avt_bn_finalize_rep": (_I, [_P, _L, _L, _I, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P]),
    "avt_conv3d_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "avt_video_stem_im2col": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "avt_maxpool3d_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "avt_pack3d_desc_bytes": (_Z, []),
    "avt_pack_conv3d_weights_batched": (_I, [_P, _I, _I, _I, _P]),
    "avt_pack_conv3d_weight": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "avt_repeat_rows_f32": (_I, [_P, _P, _I, _I, _I, _P]),
    "avt_sum_rep_rows_f32": (_I, [_P, _P, _I, _I, _I, _P]),
    "avt_bn_apply": (_I, [_P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _P]),
    "avt_bn_bwd_workspace": (_Z, [_L, _I]),
    "avt_bn_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P]),
    "avt_bn_relu_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P]),
    "avt_stem_bn_relu_maxpool_fwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "avt_stem_maxpool_bn_relu_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "avt_maxpool3s2_fwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "avt_maxpool3s2_bwd": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
    "avt_audio_pool_norm_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _P]),
    "avt_audio_pool_norm_bwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "avt_hardway_save_floats": (_Z, [_I]),
    "avt_hardway_fwd": (_I, [_P, _P, _I, _I, _I, _F, _F, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "avt_hardway_ce": (_I, [_P, _I, _I, _F, _P, _P, _P]),
    "avt_hardway_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I,
                             _P]),
    "avt_hardway_bwd_ex": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                _P, _P, _I, _P, _P]),
    "avt_hardway_bwd_ws_floats": (_Z, [_I, _I]),
    "avt_hardway_attention_fwd": (_I, [_P, _P, _I, _I, _I, _F, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "avt_hardway_attention_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _F, _P, _P, _P, _P, _P, _P]),
    "avt_twoview_loss": (_I, [_P, _P, _P, _P, _I, _I, _I, _F, _P, _P, _P, _P]),
    "avt_loss_workspace_floats": (_Z, [_L, _L]),
    "avt_propagation_loss": (_I, [_P, _I, _I, _I, _P, _P, _P, _P]),
    "avt_npratio_loss": (_I, [_P, _I, _I, _I, _P, _P, _P, _P]),
    "avt_flip_l1_loss": (_I, [_P, _P, _L, _I, _P, _P, _P, _P, _P]),
    "avt_localize_ciou": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "avt_pair_ciou": (_I, [_P, _I, _I, _P, _P]),
    "avt_spectrogram_segments": (_I, [_L, _I]),
    "avt_spectrogram": (_I, [_P, _I, _L, _I, _F, _P, _P]),
    "avt_frames_transform": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P]),
    "avt_adam_step": (_I, [_P, _P, _P, _P, _L, _F, _F, _F, _F, _F, _F, _I, _P]),
    "avt_adam_step_dev": (_I, [_P, _P, _P, _P, _L, _F, _P, _P, _P, _P]),
    "avt_adam_prep_dev": (_I, [_P, _P, _P, _P]),
    "avt_adam_apply_dev": (_I, [_P, _P, _P, _P, _L, _F, _P, _P]),
    "avt_pack_conv_weights_part": (_I, [_P, _I, _L, _I, _P]),
    "avt_pack_conv_weight": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "avt_pack_desc_bytes": (_Z, []),
    "avt_pack_conv_weights_batched": (_I, [_P, _I, _L, _P]),
    "avt_nchw_to_nhwc_bf16": (_I, [_P, _P, _I, _I, _I, _I, _I, _P]),
    "avt_ncthw_to_nhwc_bf16": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "avt_nhwc_bf16_to_nchw": (_I, [_P, _P, _I, _I, _I, _P]),
}

_lock = threading.Lock()
_lib = None


INCLUDE = os.path.join(os.path.dirname(PKG_DIR), "include")
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + INCLUDE, "-shared"]
HASH_PATH = LIB_PATH + ".sha256"


def source_hash() -> str:
    """sha256 over every csrc/*.hip, csrc/*.h, include/*.h and the compile flags: the identity of a
    build.  build() records it next to libavt.so; lib() refuses a library whose record differs
    (a stale .so shipped with newer sources)."""
    import hashlib

    h = hashlib.sha256(" ".join([f for f in HIPCC_FLAGS if not f.startswith("-I")] + SOURCES).encode())
    inc = INCLUDE
    files = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h")))
    if os.path.isdir(inc):
        files += sorted(os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h"))
    for p in files:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _recorded_hash() -> str:
    try:
        with open(HASH_PATH) as f:
            return f.read().strip()
    except OSError:
        return ""


def build(verbose: bool = False, force: bool = False) -> str:
    """Compile csrc/*.hip for gfx950 into libavt.so (in-tree); rebuilds whenever the sources' hash
    differs from the one recorded at the last build."""
    digest = source_hash()
    if not force and os.path.exists(LIB_PATH) and _recorded_hash() == digest:
        return LIB_PATH
    import concurrent.futures
    import tempfile

    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = LIB_PATH + ".tmp"
    with tempfile.TemporaryDirectory(prefix="avt_build_") as bdir:
        def compile_one(src):
            obj = os.path.join(bdir, os.path.splitext(src)[0] + ".o")
            cmd = [hipcc] + HIPCC_FLAGS[:-1] + ["-c", os.path.join(CSRC, src), "-o", obj]  # no -shared
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True, cwd=CSRC)
            return obj

        jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
        with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
            objs = list(ex.map(compile_one, SOURCES))
        cmd = [hipcc] + HIPCC_FLAGS + ["-o", tmp] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(tmp, LIB_PATH)
    with open(HASH_PATH, "w") as f:
        f.write(digest + "\n")
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LOAD_PATH):
                raise RuntimeError(f"libavt.so not built ({LOAD_PATH}); run __graft_entry__.build()")
            if LOAD_PATH == LIB_PATH and _recorded_hash() != source_hash():
                raise RuntimeError(f"{LIB_PATH} was not built from the current csrc/ sources (hash record "
                                   f"{HASH_PATH} differs); run __graft_entry__.build()")
            h = ctypes.CDLL(LOAD_PATH)
            for name, (res, args) in SIGNATURES.items():
                if LOAD_PATH != LIB_PATH and not hasattr(h, name):
                    continue  # an older A/B build
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _lib = h
    return _lib


def call(name: str, *args) -> int:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().avt_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed ({rc}): {msg}")
    return rc


def query(name: str, *args):
    return getattr(lib(), name)(*args)
