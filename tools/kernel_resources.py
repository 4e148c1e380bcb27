"""Per-kernel resources of a built libgossip_hip.so (gfx950 code object notes): LDS bytes, VGPRs,
SGPRs, scratch and spills, for the kernels whose name matches a pattern.

    python3 tools/kernel_resources.py [LIB] [PATTERN]     # e.g. ... lib/libgossip_hip.so quiet_x
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def notes_of(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "gfx950.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                              text=True).stdout


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "cop5615-gossip_protocol_amd", "lib",
                                                             "libgossip_hip.so")
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    notes = notes_of(lib)
    # one metadata block per kernel: split at each "- .agpr_count" / ".args" start is fragile; use .name order
    blocks = re.split(r"\n\s*- \.", notes)
    for b in blocks:
        m = re.search(r"^\s*\.name:\s+(\S+)", b, re.M)
        if not m or not m.group(1).startswith("_Z"):
            continue
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        if pat not in name:
            continue

        def val(key):
            x = re.search(rf"\.{key}:\s+(\d+)", b)
            return int(x.group(1)) if x else -1

        print(f"{name[:90]:90s} lds={val('group_segment_fixed_size'):6d} vgpr={val('vgpr_count'):4d} "
              f"sgpr={val('sgpr_count'):4d} scratch={val('private_segment_fixed_size')} "
              f"spill={val('vgpr_spill_count')}/{val('sgpr_spill_count')}")


if __name__ == "__main__":
    main()
