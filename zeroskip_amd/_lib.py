"""ctypes binding of libzscrc.so (the C ABI of include/zscrc.h)."""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZSCRC_LIB_PATH: another build of the same ABI (A/B timing runs of two builds)
LIB_PATH = os.environ.get("ZSCRC_LIB_PATH") or os.path.join(_HERE, "libzscrc.so")

# library defaults of zscrc_set_teams(g1_max, g16_max) (zscrc_api.cpp g_g1_max, g_g16_max)
DEFAULT_TEAMS = (640, 1 << 20)
QTEAM_DEFAULT = 1  # zscrc_api.cpp g_qteam

_u32, _u64, _vp, _sz, _int = (ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                              ctypes.c_size_t, ctypes.c_int)

# name -> (restype, argtypes); mirrors include/zscrc.h
SIGNATURES = {
    "crc32c_init": (None, []),
    "crc32c_sw": (_u32, [_u32, _vp, _sz]),
    "crc32c_hw": (_u32, [_u32, _vp, _sz]),
    "crc32c": (_u32, [_u32, _vp, _sz]),
    "crc32c_map": (_u32, [ctypes.c_char_p, ctypes.c_uint]),
    "crc32c_cstring": (_u32, [_vp]),
    "crc32c_buf": (_u32, [ctypes.c_char_p]),
    "crc32c_iovec": (_u32, [_vp, _int]),
    "crc32c_combine": (_u32, [_u32, _u32, _u64]),
    "zscrc_shift": (_u32, [_u32, _u64]),
    "zscrc_device_batch": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint, _vp]),
    "zscrc_device_fixed": (_int, [_vp, _u64, _u64, _u32, _vp, _sz, ctypes.c_uint, _vp]),
    "zscrc_device_fixed_multi": (_int, [_vp, _vp, _sz, _u64, _u64, _u32, _sz, ctypes.c_uint, _vp]),
    "zscrc_span_scratch_bytes": (_sz, [_u64]),
    "zscrc_device_span": (_int, [_vp, _u64, _u32, _vp, _vp, ctypes.c_uint, _vp]),
    "zscrc_device_spans": (_int, [_vp, _vp, _vp, _vp, _sz, ctypes.c_uint, _vp]),
    "zscrc_device_mismatch_rows": (_int, [_vp, _vp, _vp, _vp, _u64, _sz, _vp, _vp, _u32, _vp]),
    "zscrc_host_batch": (_int, [_vp, _vp, _vp, _vp, _vp, _sz]),
    "zscrc_last_error": (ctypes.c_char_p, []),
    "zscrc_stats": (None, [_vp]),
    "zscrc_set_gpu_min": (None, [_u64]),
    "zscrc_gpu_min": (_u64, [_int]),
    "zscrc_set_gpu_min_pair": (None, [_u64, _u64]),
    "zscrc_warmup": (_int, []),
    "zscrc_set_teams": (None, [_u64, _u64]),
    "zscrc_set_small_team": (None, [_int]),
    "zscrc_team_for": (_int, [_u64, _u64]),
    "zscrc_set_xteam": (None, [_int, _u64]),
    "zscrc_xteam_for": (_int, [_u64, _u64]),
    "zscrc_set_opt": (None, [ctypes.c_uint]),
    "zscrc_set_qteam": (None, [_int]),
    "zscrc_set_xdeal": (ctypes.c_uint, [ctypes.c_uint]),
    "zscrc_fixed_kernel": (ctypes.c_char_p, [_vp, _u64, _u64, _sz]),
    "zscrc_set_prefetch": (None, [_int, _int]),
    "zscrc_diag_stream_read": (_int, [_vp, _u64, _vp, _int, _vp]),
    "zscrc_diag_wave_times": (_int, [_vp]),
    "zscrc_diag_classify_times": (_int, [_vp]),
    "zscrc_device_count": (_int, []),
    "zscrc_zs_walk": (_int, [_vp, _u64, _vp, _vp, _sz, _vp, _vp]),
    "zscrc_zs_packed_spans": (_int, [_vp, _u64, _vp, _vp]),
    "zscrc_zs_header_crc": (_int, [_vp, _u64, _vp, _vp]),
    "zscrc_zs_dotzsdb_crc": (_int, [_vp, _u64, _vp, _vp]),
    "zscrc_device_verify_commits": (_int, [_vp, _u64, _vp, _vp, _sz, _vp, _vp, _vp]),
    "zscrc_device_verify_commits_seeded": (_int, [_vp, _u64, _vp, _vp, _vp, _sz, _vp, _vp, _vp]),
    "zscrc_device_verify_commits_bounded": (_int, [_vp, _u64, _vp, _vp, _vp, _sz, _u64, _vp, _vp, _vp]),
    "zscrc_device_write_commits_bounded": (_int, [_vp, _u64, _vp, _vp, _sz, _u64, _vp, _vp, _vp]),
    "zscrc_device_batch_bounded": (_int, [_vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint, _u64, _vp]),
    "zscrc_zs_verify_image": (_int, [_vp, _u64, _int, _vp]),
    "zscrc_device_write_commits": (_int, [_vp, _u64, _vp, _vp, _sz, _vp, _vp, _vp]),
    "zscrc_stream_open": (_int, [_vp, _u32, _u64, ctypes.c_uint]),
    "zscrc_stream_update": (_int, [_vp, _vp, _sz]),
    "zscrc_stream_final": (_int, [_vp, _vp]),
    "zscrc_zs_consistent": (_int, [ctypes.c_char_p, _vp]),
    "zscrc_zs_verify_files": (_int, [_vp, _vp, _vp, _sz, _int, _vp]),
    "zscrc_pack_open": (_int, [_vp, ctypes.c_char_p, ctypes.c_char_p, _u32, _u32, _u64, ctypes.c_uint]),
    "zscrc_pack_add": (_int, [_vp, _vp, _u64, _vp, _u64]),
    "zscrc_pack_add_batch": (_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz]),
    "zscrc_pack_close": (_int, [_vp, _vp]),
    "zscrc_abi_version": (_int, []),
    "zscrc_cpass_create": (_int, [_vp, _vp]),
    "zscrc_cpass_run": (_int, [_vp, _vp, _vp]),
    "zscrc_cpass_run_timed": (_int, [_vp, _vp, _vp, _vp, _vp]),
    "zscrc_cpass_submit": (_int, [_vp, _vp, _vp, _vp, ctypes.c_int]),
    "zscrc_cpass_collect": (_int, [_vp, ctypes.c_int, _vp]),
    "zscrc_cpass_set_row": (_int, [_vp, _vp]),
    "zscrc_cpass_submit_row": (_int, [_vp, _vp, _vp, _vp, _vp]),
    "zscrc_cpass_destroy": (None, [_vp]),
    "zscrc_device_verify_commits_verdict": (_int, [_vp, _u64, _vp, _vp, _vp, _sz, _u64, _vp, _vp, _sz, _vp]),
    "zscrc_pack_abort": (_int, [_vp]),
    "zscrc_zs_records": (_int, [_vp, _u64, _int, _vp, _sz, _vp]),
    "zscrc_zs_dotzsdb_build": (_int, [_u64, ctypes.c_char_p, _u32, _vp]),
    "zscrc_zs_repack": (_int, [ctypes.c_char_p, ctypes.c_uint, _int, _vp]),
    "zscrc_set_devices": (_int, [_vp, _int]),
    "zscrc_files_devices": (_int, [_vp, _int]),
    "zscrc_release_cache": (None, []),
    "zscrc_device_commit_crcs_bounded": (_int, [_vp, _u64, _vp, _vp, _sz, _u64, _vp, _vp, _vp]),
    "zscrc_zs_fill_commits": (_int, [_vp, _u64, _vp, _vp, _sz, _u64, _int, _vp]),
    "zscrc_device_verify_commits_verdict_range": (_int, [_vp, _u64, _vp, _vp, _vp, _sz, _u64, _u64, _vp, _vp, _sz,
                                                         _vp]),
}
ABI_VERSION = 4  # include/zscrc.h ZSCRC_ABI_VERSION

ZSCRC_RAW = 1
LEN_UNBOUNDED = (1 << 64) - 1  # ZSCRC_LEN_UNBOUNDED
ZSCRC_STREAM_NOCOPY = 1

_lib = None


class ZscrcError(RuntimeError):
    pass


def build_library(force: bool = False) -> str:
    """Compile libzscrc.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    args = ["make", "-s", "-C", _HERE] + (["-B"] if force else [])
    subprocess.check_call(args)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C {_HERE}` "
                "(there is no CPU fallback for the GPU engine)")
        L = ctypes.CDLL(LIB_PATH)
        # an older build under ZSCRC_LIB_PATH (A/B timing runs) may lack the
        # newer entry points; the in-tree library must have them all
        other = bool(os.environ.get("ZSCRC_LIB_PATH"))
        for name, (res, args) in SIGNATURES.items():
            if other and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if not other and L.zscrc_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH}: ABI {L.zscrc_abi_version()}, this binding expects {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int, what: str = "libzscrc") -> None:
    if rc != 0:
        msg = lib().zscrc_last_error()
        raise ZscrcError(f"{what} failed with status {rc}: {msg.decode() if msg else ''}")


def stats() -> list[int]:
    a = (ctypes.c_uint64 * 4)()
    lib().zscrc_stats(a)
    return list(a)
