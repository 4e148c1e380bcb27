"""ctypes binding of libgossip_hip.so (include/gossip_hip.h).

The product path: there is no CPU fallback.  If the HIP library is missing or fails to load,
import raises — the CPU oracle lives in oracle/ and is test infrastructure only.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# GP_LIB (tuning only): load a variant build, e.g. lib_<name>/ from tools/variants/build.sh
LIB_PATH = os.path.join(PKG_ROOT, os.environ.get("GP_LIB", "lib"), "libgossip_hip.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "gossip_hip.h")

ABI_VERSION = 8
TOPOLOGIES = {"line": 0, "full": 1, "2D": 2, "Imp3D": 3, "3D": 4}
ALGOS = {"gossip": 0, "push-sum": 1}
FLAG_KERNEL_TIMING = 1
FLAG_GENERIC = 2
FLAG_USE_STREAM = 4
FLAG_ONE_DEVICE = 8
FLAG_GROUP = 16
FLAG_QUIET_WAVES = 32
FLAG_GOSSIP_TALLY = 64
FLAG_FULL_PLAN = 128
FLAG_TIGHT_TIERS = 256
FLAG_TALLY_FALLBACKS = 512
FLAG_PIECES = 1024
FLAG_FORCE_PIECES = 2048
FLAG_ONE_ROUND = 4096
ERRORS = {-1: "GP_EINVAL", -2: "GP_ENOMEM", -3: "GP_EHIP", -4: "GP_ESTATE", -5: "GP_EOVERFLOW", -6: "GP_ERCCL"}


class Config(C.Structure):
    _fields_ = [("n_arg", C.c_int64), ("topology", C.c_int32), ("algo", C.c_int32),
                ("seed", C.c_uint64), ("delta", C.c_double), ("gossip_threshold", C.c_int32),
                ("term_init", C.c_int32), ("term_limit", C.c_int32), ("device", C.c_int32),
                ("flags", C.c_int32), ("num_gpus", C.c_int32), ("stream", C.c_void_p)]


class Layout(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("actors", C.c_int64), ("grid", C.c_int64),
                ("leader", C.c_int64), ("participants", C.c_int64), ("links", C.c_int64),
                ("device_bytes", C.c_int64)]


class Status(C.Structure):
    _fields_ = [("round", C.c_int64), ("completed", C.c_int64), ("converged", C.c_int32),
                ("pad", C.c_int32), ("sum_s", C.c_double), ("sum_w", C.c_double),
                ("device_ms", C.c_double)]


class KStats(C.Structure):
    _fields_ = [("launches", C.c_int64), ("total_ms", C.c_double), ("avg_ms", C.c_double),
                ("bytes_per_launch", C.c_double), ("kernel", C.c_char * 64),
                ("aux_avg_ms", C.c_double), ("aux_kernel", C.c_char * 64), ("work_per_launch", C.c_double)]


class ShardLayout(C.Structure):
    _fields_ = [("lo", C.c_int64), ("hi", C.c_int64), ("halo", C.c_int64),
                ("send_total", C.c_int64), ("recv_total", C.c_int64)]


class ShardStats(C.Structure):
    _fields_ = [("plan_changes", C.c_int64), ("restores", C.c_int64), ("send_bytes", C.c_int64),
                ("recv_bytes", C.c_int64), ("restore_round", C.c_int64), ("bytes_sent", C.c_int64),
                ("list_rounds", C.c_int64), ("bin_rounds", C.c_int64)]


EXPORTS = ["gp_abi_version", "gp_sizes", "gp_create", "gp_reset", "gp_step", "gp_read_gossip",
           "gp_read_pushsum", "gp_read_messages", "gp_read_trace", "gp_neighbors",
           "gp_kernel_stats", "gp_partition", "gp_create_shard", "gp_shard_plan", "gp_shard_round",
           "gp_shard_deliver", "gp_shard_sync", "gp_shard_stats", "gp_shard_pieces", "gp_shard_round_piece",
           "gp_shard_plan_piece", "gp_destroy", "gp_last_error"]


class GossipError(RuntimeError):
    pass


_lib = None


def load():
    """Load libgossip_hip.so (raises if absent: build it with `make -C cop5615-gossip_protocol_amd`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GossipError(f"HIP engine not built: {LIB_PATH} missing (run __graft_entry__.build())")
    # One HIP runtime per process: torch bundles its own libamdhip64 / libhsa-runtime64 with the
    # same sonames as /opt/rocm's.  Loaded first, they satisfy this library's dependencies, so
    # kernels, streams and RCCL buffers all live in torch's runtime.  Loading ours first would
    # bring a second runtime into the process, and one of the two then finds no device.
    import torch  # noqa: F401

    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.gp_abi_version.restype = C.c_int
    L.gp_sizes.argtypes = [C.c_int64, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.gp_create.argtypes = [C.POINTER(Config), C.POINTER(Layout), C.POINTER(C.c_void_p)]
    L.gp_reset.argtypes = [P]
    L.gp_step.argtypes = [P, C.c_int64, C.POINTER(Status)]
    L.gp_read_gossip.argtypes = [P, C.c_int64, C.c_int64, P, P]
    L.gp_read_pushsum.argtypes = [P, C.c_int64, C.c_int64, P, P, P]
    L.gp_read_messages.argtypes = [P, C.c_int64, C.c_int64, P, P, P]
    L.gp_read_trace.argtypes = [P, C.c_int64, C.c_int64, P]
    L.gp_neighbors.argtypes = [P, C.c_int64, P, C.c_int32]
    L.gp_kernel_stats.argtypes = [P, C.POINTER(KStats), C.c_int32]
    L.gp_partition.argtypes = [C.c_int64, C.c_int32, C.c_int32, P]
    L.gp_create_shard.argtypes = [C.POINTER(Config), C.c_int32, C.c_int32, C.POINTER(Layout),
                                  C.POINTER(ShardLayout), C.POINTER(C.c_void_p)]
    L.gp_shard_plan.argtypes = [P, P, P]
    L.gp_shard_round.argtypes = [P, P]
    L.gp_shard_deliver.argtypes = [P, P]
    L.gp_shard_sync.argtypes = [P, C.POINTER(Status)]
    L.gp_shard_stats.argtypes = [P, C.POINTER(ShardStats)]
    L.gp_shard_pieces.argtypes = [P]
    L.gp_shard_round_piece.argtypes = [P, P, C.c_int32]
    L.gp_shard_plan_piece.argtypes = [P, C.c_int32, P, P, P]
    L.gp_destroy.argtypes = [P]
    L.gp_destroy.restype = None
    L.gp_last_error.restype = C.c_char_p
    if L.gp_abi_version() != ABI_VERSION:
        raise GossipError(f"ABI mismatch: library {L.gp_abi_version()} != {ABI_VERSION}")
    _lib = L
    return L


def check(rc: int):
    if rc != 0:
        msg = load().gp_last_error().decode(errors="replace")
        raise GossipError(f"{ERRORS.get(rc, rc)}: {msg}")
