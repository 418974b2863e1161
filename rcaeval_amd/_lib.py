"""ctypes binding of ``libpcgpu.so`` (declared in ``include/pcgpu.h``).

The library is built in-tree (``rcaeval_amd/libpcgpu.so``) by ``__graft_entry__.build()`` /
``make -C rcaeval_amd/csrc``. There is no CPU fallback: if the library is missing or no
GPU is visible, every engine entry point raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCG_LIB_PATH: an A/B build variant (tools/variant_bench.sh) loaded instead of the in-tree library,
# so no script ever overwrites rcaeval_amd/libpcgpu.so
LIB_PATH = os.environ.get("PCG_LIB_PATH") or os.path.join(_HERE, "libpcgpu.so")

PCG_OK = 0
PCG_ERR_INVALID = -1
PCG_ERR_OOM = -2
PCG_ERR_HIP = -3
PCG_ERR_SINGULAR = -4
PCG_ERR_DOMAIN = -5
PCG_ERR_RCCL = -6
PCG_ERR_OVERFLOW = -7
PCG_ERR_PEER = -8

PCG_FLAG_FULL_P = 0x1
PCG_FLAG_RECORD = 0x2
PCG_FLAG_EXACT_ALL = 0x4

PCG_MAX_LEVELS = 32
PCG_ABI_VERSION = 4         # include/pcgpu.h; checked against the library by load()
PCG_RM_STATUS = 64          # status bytes after the n*n removal flags (pcgpu.h)
PCG_MAX_DEPTH = 12
PCG_MAX_LEVEL_DEPTH = 30

# pcg_stats.driver
PCG_DRIVER_LEVELS = 0
PCG_DRIVER_SMALL = 1
PCG_DRIVER_SMALL_RERUN = 2
DRIVER_NAMES = {PCG_DRIVER_LEVELS: "levels", PCG_DRIVER_SMALL: "small", PCG_DRIVER_SMALL_RERUN: "small_rerun"}

# pcg_set_tuning keys (include/pcgpu.h PCG_TUNE_*), by their environment names without "PCG_"
TUNE_KEYS = {
    "SMALL": 0, "SMALL_QCAP": 1, "LDS_DEEP": 2, "LDS_SPILL_MIN": 3, "WAVE_LO": 4, "SCREEN_MASK": 5,
    "NODE_BLOCKS": 6, "EXPORT_INLINE": 7, "NB": 8, "NBW": 9, "HOST_TRACE": 10, "K1_I8": 11, "K1_CRT": 12,
    "K1_CRT_MINN": 13, "K1_CRT_BITS": 14, "K1_CRT_KS": 15, "K1_I8_KS": 16, "K1_SUPER_ORDER": 17,
    "L1Z": 18,
}

I64 = ctypes.c_int64
I32 = ctypes.c_int32
P = ctypes.c_void_p
D = ctypes.c_double


class PcgStats(ctypes.Structure):
    _fields_ = [
        ("tests", I64 * PCG_MAX_LEVELS),
        ("calls", I64 * PCG_MAX_LEVELS),
        ("indep", I64 * PCG_MAX_LEVELS),
        ("exact", I64 * PCG_MAX_LEVELS),
        ("near_alpha", I64 * PCG_MAX_LEVELS),
        ("edges_after", I64 * PCG_MAX_LEVELS),
        ("max_degree", I32 * PCG_MAX_LEVELS),
        ("level_ms", D * PCG_MAX_LEVELS),
        ("kernel_ms", D * PCG_MAX_LEVELS),
        ("levels", I32),
        ("error", I32),
        ("screened", I64 * PCG_MAX_LEVELS),
        ("driver", I32),
        ("driver_pad", I32),
    ]

    def as_dict(self) -> dict:
        L = self.levels
        return {
            "levels": L,
            "error": self.error,
            "tests": list(self.tests[:L]),
            "calls": list(self.calls[:L]),
            "indep": list(self.indep[:L]),
            "exact": list(self.exact[:L]),
            "near_alpha": list(self.near_alpha[:L]),
            "edges_after": list(self.edges_after[:L]),
            "max_degree": list(self.max_degree[:L]),
            "level_ms": list(self.level_ms[:L]),
            "kernel_ms": list(self.kernel_ms[:L]),
            "screened": list(self.screened[:L]),
            "driver": DRIVER_NAMES.get(self.driver, str(self.driver)),
        }


class PcgRecord(ctypes.Structure):
    _fields_ = [("a", I32), ("b", I32), ("d", I32), ("s", I32 * PCG_MAX_DEPTH), ("p", D)]


# (name, restype, argtypes) — exactly the exports of include/pcgpu.h
SIGNATURES = [
    ("pcg_abi_info", I32, [ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(I32)]),
    ("pcg_create", I32, [ctypes.c_int, ctypes.POINTER(P)]),
    ("pcg_destroy", I32, [P]),
    ("pcg_last_error", ctypes.c_char_p, [P]),
    ("pcg_set_stream", I32, [P, P]),
    ("pcg_set_capacity", I32, [P, I64, I64]),
    ("pcg_set_record_sample", I32, [P, I64, I64]),
    ("pcg_set_tuning", I32, [P, ctypes.c_int, I64]),
    ("pcg_get_tuning", I32, [P, ctypes.c_int, ctypes.POINTER(I64)]),
    ("pcg_k1_plan_signature", I32, [P, I64, I64, ctypes.POINTER(I64)]),
    ("pcg_corr", I32, [P, P, I64, I64, I64, P, I64]),
    ("pcg_corr_shard_rows", I32, [I64, ctypes.c_int, ctypes.POINTER(I64)]),
    ("pcg_corr_shard_bytes", I32, [P, I64, I64, ctypes.c_int, ctypes.POINTER(I64)]),
    ("pcg_corr_shard", I32, [P, P, I64, I64, I64, ctypes.c_int, ctypes.c_int, P]),
    ("pcg_corr_shard_finish", I32, [P, P, I64, I64, ctypes.c_int, P, I64]),
    ("pcg_skeleton", I32, [P, P, I64, I64, I64, D, ctypes.c_int, ctypes.c_int, P, ctypes.POINTER(PcgStats)]),
    ("pcg_pc_skeleton", I32, [P, P, I64, I64, I64, P, I64, D, ctypes.c_int, ctypes.c_int, P,
                          ctypes.POINTER(PcgStats)]),
    ("pcg_degrees", I32, [P, P, I64]),
    ("pcg_sepset_count", I32, [P, ctypes.POINTER(I64), ctypes.POINTER(I32)]),
    ("pcg_sepset_export", I32, [P, P, P, I64]),
    ("pcg_sepset_export_device", I32, [P, P, P, I64]),
    ("pcg_set_sepset_buffers", I32, [P, P, P, I64]),
    ("pcg_sepset_target", I32, [P, ctypes.POINTER(I32), ctypes.POINTER(I64)]),
    ("pcg_record_count", I32, [P, ctypes.POINTER(I64), ctypes.POINTER(I64)]),
    ("pcg_record_export", I32, [P, P, I64, P, I64]),
    ("pcg_skeleton_init", I32, [P, P, I64, I64, I64, D, ctypes.c_int, P]),
    ("pcg_level_begin", I32, [P, ctypes.c_int, ctypes.POINTER(I64), ctypes.POINTER(I32), ctypes.POINTER(P)]),
    ("pcg_level_run", I32, [P, I64, I64]),
    ("pcg_level_end", I32, [P, ctypes.POINTER(PcgStats)]),
    ("pcg_level_chunk_work", I32, [P, P, I64]),
    ("pcg_level_split", I32, [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(I64), ctypes.POINTER(I64)]),
    ("pcg_set_removal_buffer", I32, [P, P, I64]),
    ("pcg_level_packed_words", I32, [I64, ctypes.POINTER(I64)]),
    ("pcg_level_pack", I32, [P, P, ctypes.c_int]),
    ("pcg_level_merge", I32, [P, P, ctypes.c_int]),
    ("pcg_set_world_size", I32, [P, ctypes.c_int]),
    ("pcg_set_narrow_degree", I32, [P, ctypes.c_int]),
    ("pcg_set_screen_precision", I32, [P, ctypes.c_int]),
    ("pcg_set_screen_capacity", I32, [P, ctypes.c_int64]),
    ("pcg_comm_unique_id", I32, [P, I64]),
    ("pcg_comm_init", I32, [P, P, ctypes.c_int, ctypes.c_int]),
    ("pcg_comm_destroy", I32, [P]),
    ("pcg_comm_group_create", I32, [ctypes.c_int, D, ctypes.POINTER(P)]),
    ("pcg_comm_group_destroy", I32, [P]),
    ("pcg_comm_group_stats", I32, [P, ctypes.POINTER(I64), ctypes.POINTER(I64), ctypes.POINTER(I32)]),
    ("pcg_comm_init_group", I32, [P, P, ctypes.c_int]),
    ("pcg_corr_sharded", I32, [P, P, I64, I64, I64, P, I64]),
    ("pcg_skeleton_sharded", I32, [P, P, I64, I64, I64, D, ctypes.c_int, ctypes.c_int, P, ctypes.POINTER(PcgStats)]),
    ("pcg_pagerank_dense", I32, [P, P, I64, I64, D, ctypes.c_int, D, P]),
    ("pcg_pagerank_csr", I32, [P, P, P, P, I64, I64, D, ctypes.c_int, D, P]),
    ("pcg_random_walk", I32, [P, P, I64, I64, I64, I64, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.c_uint64, ctypes.c_uint64, P]),
    ("pcg_orient", I32, [I64, P, P, P, I64, ctypes.c_int, P]),
    ("pcg_uc_candidates", I32, [I64, P, P, P, I64, P, I64, ctypes.POINTER(I64)]),
    ("pcg_orient_triples", I32, [I64, P, P, I64, P]),
    ("pcg_orient_bk", I32, [I64, P, P, P, I64, ctypes.c_int, P, P, I64, P, P, P]),
    ("pcg_set_forbidden_pairs", I32, [P, P]),
    ("pcg_fisherz_batch", I32, [P, P, I64, I64, I64, P, I32, I64, P, P]),
    ("pcg_chisq_batch", I32, [P, P, I64, I64, P, P, I32, I64, ctypes.c_int, I64, P, P, P]),
]

_lib = None


class EngineUnavailable(RuntimeError):
    """The HIP engine library is missing or unusable (no silent CPU fallback exists)."""


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C rcaeval_amd/csrc` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    check_abi(lib)
    _lib = lib
    return lib


def abi_info(lib) -> tuple:
    """(sizeof(pcg_stats), sizeof(pcg_record), PCG_ABI_VERSION) as the library was built."""
    sb, rb, ver = I64(), I64(), I32()
    lib.pcg_abi_info(ctypes.byref(sb), ctypes.byref(rb), ctypes.byref(ver))
    return sb.value, rb.value, ver.value


def check_abi(lib, stats_cls=None, record_cls=None) -> None:
    """Refuse a library whose struct layouts or ABI version differ from these bindings (a
    stale .so, or a header change the ctypes structs did not follow)."""
    stats_cls = stats_cls or PcgStats
    record_cls = record_cls or PcgRecord
    sb, rb, ver = abi_info(lib)
    mine = (ctypes.sizeof(stats_cls), ctypes.sizeof(record_cls), PCG_ABI_VERSION)
    if (sb, rb, ver) != mine:
        raise EngineUnavailable(
            f"{LIB_PATH}: ABI mismatch (library sizeof(pcg_stats)={sb}, sizeof(pcg_record)={rb}, "
            f"version {ver}; bindings {mine[0]}, {mine[1]}, version {mine[2]}): rebuild the library "
            "or update rcaeval_amd/_lib.py with include/pcgpu.h")


class PcgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[pcgpu {code}] {msg}")
        self.code = code


def check(handle, rc: int, what: str) -> int:
    if rc < 0:
        msg = load().pcg_last_error(handle)
        msg = msg.decode() if msg else what
        if rc in (PCG_ERR_SINGULAR, PCG_ERR_DOMAIN):
            # causal-learn raises ValueError here [U]; @rca turns it into dummy ranks.
            raise ValueError(msg)
        raise PcgError(rc, f"{what}: {msg}")
    return rc
