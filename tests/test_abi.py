"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol the header
declares, size arithmetic matches the oracle, and calls that need a GPU fail cleanly."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from gossip_amd import _abi, sizes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(_abi.HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gp_\w+)\s*\(", text, re.M)))


def test_header_declares_exports():
    assert header_functions() == sorted(_abi.EXPORTS)


def test_library_exports_every_symbol():
    L = _abi.load()
    for name in header_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (gp_\w+)$", out, re.M))
    assert set(header_functions()) <= exported


def test_abi_version():
    assert _abi.load().gp_abi_version() == _abi.ABI_VERSION


@pytest.mark.parametrize("topo", ["line", "full", "2D", "Imp3D", "3D"])
@pytest.mark.parametrize("n", [1, 2, 7, 8, 20, 133, 200, 488, 5831, 100000, 10000000, 1000000000])
def test_sizes_match_oracle(topo, n):
    assert sizes(n, topo) == oracle.sizes(n, topo)


def test_sizes_reject_bad_input():
    with pytest.raises(_abi.GossipError):
        sizes(0, "line")
    with pytest.raises(ValueError):
        from gossip_amd import Simulator
        Simulator(10, "imp3D", "gossip")  # case-sensitive (program.fs:267)


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from gossip_amd import Simulator
    with pytest.raises(_abi.GossipError, match="GP_EHIP"):
        Simulator(100, "Imp3D", "push-sum")


def test_cli_argument_contract():
    exe = os.path.join(ROOT, "cop5615-gossip_protocol_amd", "lib", "gossip")
    r = subprocess.run([exe, "100", "line", "gosip"], capture_output=True, text=True)
    assert r.returncode == 2 and r.stdout.strip() == "Invalid:Please enter a proper protocol or topology"
    r = subprocess.run([exe, "100", "2D", "x"], capture_output=True, text=True)
    assert r.stdout.strip() == "Invalid: Please enter a proper protocol or topology"  # program.fs:265
    r = subprocess.run([exe, "100", "imp3D", "gossip"], capture_output=True, text=True)
    assert r.returncode == 2
    r = subprocess.run([exe, "100"], capture_output=True, text=True)
    assert r.returncode == 2
    r = subprocess.run([exe, "100", "line", "gossip", "--mode", "async"], capture_output=True, text=True)
    assert r.returncode == 2 and "--mode async" in r.stderr  # only the round engine is built
    r = subprocess.run([exe, "100", "line", "gossip", "--quiet"], capture_output=True, text=True)
    assert r.returncode == 2  # unknown option


def test_kstats_struct_layout():
    """gp_kstats as the header lays it out (ABI 4 appended work_per_launch), field by field."""
    import ctypes as C

    text = open(_abi.HEADER).read()
    body = re.search(r"typedef struct gp_kstats \{(.*?)\} gp_kstats;", text, re.S).group(1)
    names = re.findall(r"^\s*(?:int64_t|double|char)\s+(\w+)", body, re.M)
    assert names == [f[0] for f in _abi.KStats._fields_] == [
        "launches", "total_ms", "avg_ms", "bytes_per_launch", "kernel", "aux_avg_ms", "aux_kernel", "work_per_launch"]
    assert _abi.KStats.work_per_launch.offset == 168 and C.sizeof(_abi.KStats) == 176
    assert _abi.ABI_VERSION == 8 and re.search(r"#define GP_ABI_VERSION 8\b", text)


def test_shard_counters_struct_layout():
    """gp_shard_counters (ABI 5: activity tiers of the shard exchange; ABI 6 appended bytes_sent, ABI 8
    list_rounds and bin_rounds) as the header lays it out."""
    import ctypes as C

    text = open(_abi.HEADER).read()
    body = re.search(r"typedef struct gp_shard_counters \{(.*?)\} gp_shard_counters;", text, re.S).group(1)
    names = re.findall(r"^\s*int64_t\s+(\w+)", body, re.M)
    assert names == [f[0] for f in _abi.ShardStats._fields_] == [
        "plan_changes", "restores", "send_bytes", "recv_bytes", "restore_round", "bytes_sent", "list_rounds",
        "bin_rounds"]
    assert C.sizeof(_abi.ShardStats) == 64


def test_config_struct_layout():
    """gp_config as the header lays it out (ABI 3: num_gpus in the former reserved slot), so a
    P/Invoke / ctypes mirror built from the header agrees field by field."""
    import ctypes as C

    text = open(_abi.HEADER).read()
    assert "int32_t num_gpus;" in text and "reserved" not in text
    assert [f[0] for f in _abi.Config._fields_] == [
        "n_arg", "topology", "algo", "seed", "delta", "gossip_threshold", "term_init", "term_limit",
        "device", "flags", "num_gpus", "stream"]
    assert C.sizeof(_abi.Config) == 64 and _abi.Config.num_gpus.offset == 52 and _abi.Config.stream.offset == 56
    for name, val in (("GP_FLAG_ONE_DEVICE", 8), ("GP_FLAG_GROUP", 16), ("GP_ERCCL", -6)):
        assert re.search(rf"{name}\s*=\s*{val}\b", text), name
    assert (_abi.FLAG_ONE_DEVICE, _abi.FLAG_GROUP, _abi.ERRORS[-6]) == (8, 16, "GP_ERCCL")


def test_library_loads_rccl_lazily():
    """Multi-GPU lives behind the ABI: the library itself drives RCCL (ncclCommInitAll, grouped
    ncclSend / ncclRecv) rather than leaving the exchange to the host, but opens it only when a
    multi-device group is created, so the one-GPU engine needs no RCCL install."""
    out = subprocess.run(["readelf", "-d", _abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl" not in out
    strings = open(_abi.LIB_PATH, "rb").read()
    for sym in (b"librccl.so.1", b"ncclCommInitAll", b"ncclSend", b"ncclRecv", b"ncclGroupStart", b"ncclGroupEnd"):
        assert sym in strings, sym


ASAN_EXE = os.path.join(ROOT, "cop5615-gossip_protocol_amd", "lib", "abi_errors_asan")


def _run_asan(*args):
    supp = os.path.join(ROOT, "tests", "native", "lsan.supp")  # the ROCm runtime's process-lifetime allocations
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", LSAN_OPTIONS=f"suppressions={supp}")
    return subprocess.run([ASAN_EXE, *args], capture_output=True, text=True, timeout=240, env=env)


def test_create_errors_free_everything_under_asan():
    """gp_create's failing paths (num_gpus 17, a missing device, numNodes 0) return their codes
    and leave nothing behind: the library's host code under AddressSanitizer / LeakSanitizer
    (tests/native/abi_errors.cpp, built by the Makefile)."""
    if not os.path.exists(ASAN_EXE):
        pytest.skip("no sanitizer build (make -C cop5615-gossip_protocol_amd check needs the host ASan runtime)")
    out = _run_asan()
    assert out.returncode == 0, out.stdout + out.stderr
    assert "LeakSanitizer" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr
    assert out.stdout.strip().endswith("done"), out.stdout


@pytest.mark.gpu
def test_group_errors_free_everything_under_asan():
    """The multi-GPU group's failure paths after shards and streams exist, and a whole group
    created, stepped and destroyed, under the host sanitizers."""
    if not os.path.exists(ASAN_EXE):
        pytest.skip("no sanitizer build (make -C cop5615-gossip_protocol_amd check needs the host ASan runtime)")
    out = _run_asan("gpu")
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert "LeakSanitizer" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-4000:]
    assert out.stdout.strip().endswith("done"), out.stdout
    print(out.stdout)


def test_flag_values_match_header():
    """The ctypes layer's gp_flags values are the header's (GP_FLAG_*)."""
    text = open(_abi.HEADER).read()
    flags = {m.group(1): int(m.group(2)) for m in re.finditer(r"GP_FLAG_(\w+)\s*=\s*(\d+)", text)}
    assert flags, "no GP_FLAG_* in the header"
    for name, value in flags.items():
        assert getattr(_abi, "FLAG_" + name) == value, name


def test_kernels_use_no_scratch(tmp_path):
    """Every gfx950 kernel of the built library keeps its state in registers and LDS: no private
    (scratch) segment and no spilled VGPRs.  (A per-lane index into the kernel arguments once made the
    compiler copy all of them to every thread's scratch: 0.5 GB of writes per launch at C4 / 8.)"""
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(f"{llvm}/clang-offload-bundler"):
        pytest.skip("no ROCm LLVM tools")
    fat, co = tmp_path / "fatbin.bin", tmp_path / "gfx950.co"
    subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", _abi.LIB_PATH], check=True)
    subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                           text=True).stdout
    names = re.findall(r"^\s*\.name:\s+(\S+)", notes, re.M)
    kernels = [n for n in names if n.startswith("_Z")]
    private = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
    spills = [int(x) for x in re.findall(r"\.vgpr_spill_count:\s+(\d+)", notes)]
    assert len(kernels) >= 40 and len(private) == len(kernels) == len(spills), (len(kernels), len(private))
    bad = [(k, p, v) for k, p, v in zip(kernels, private, spills) if p or v]
    assert not bad, bad
