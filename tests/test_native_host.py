"""Host-compiled checks of the product's shared header (no GPU needed)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fastdiv_and_presence(tmp_path):
    exe = tmp_path / "fastdiv_check"
    src = os.path.join(ROOT, "tests", "native", "fastdiv_check.cpp")
    inc = os.path.join(ROOT, "cop5615-gossip_protocol_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-I" + inc, src,
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout
