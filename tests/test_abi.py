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


def test_library_links_rccl():
    """Multi-GPU lives behind the ABI: the library itself links RCCL (ncclCommInitAll, grouped
    ncclSend / ncclRecv) rather than leaving the exchange to the host."""
    out = subprocess.run(["readelf", "-d", _abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl.so" in out
    und = subprocess.run(["nm", "-D", "--undefined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    for sym in ("ncclCommInitAll", "ncclSend", "ncclRecv", "ncclGroupStart", "ncclGroupEnd"):
        assert sym in und, sym


def test_flag_values_match_header():
    """The ctypes layer's gp_flags values are the header's (GP_FLAG_*)."""
    text = open(_abi.HEADER).read()
    flags = {m.group(1): int(m.group(2)) for m in re.finditer(r"GP_FLAG_(\w+)\s*=\s*(\d+)", text)}
    assert flags, "no GP_FLAG_* in the header"
    for name, value in flags.items():
        assert getattr(_abi, "FLAG_" + name) == value, name
