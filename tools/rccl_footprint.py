#!/usr/bin/env python3
"""rccl_footprint.py -- the LDS / register footprint of the RCCL collective kernels a process maps.

VERDICT r3 weak 5: the channel cap and the stream-K CU reservation (trainer.cpp RcclExchange) were sized
from the /opt/rocm librccl's kernel metadata, but a Python process that imports torch first binds torch's
bundled librccl.so.  This tool (CPU only, no GPU needed):

  1. loads the tnet_amd library the way bench.py does and lists the librccl / libamdhip64 files mapped
     in /proc/self/maps;
  2. for each given librccl (default: the mapped one and /opt/rocm/lib/librccl.so.1) extracts the
     .hip_fatbin section (llvm-objcopy), unbundles the gfx950 code object (clang-offload-bundler, which
     reads the compressed CCOB form) and reads the amdhsa.kernels metadata (llvm-readelf --notes);
  3. prints one JSON object: the mapped files and, per library, every collective kernel's
     group_segment_fixed_size (LDS), vgpr/agpr/sgpr counts and max_flat_workgroup_size.

usage: python3 tools/rccl_footprint.py [--out profiles/r04_rccl_footprint.json] [librccl.so ...]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mapped_runtime():
    sys.path.insert(0, os.path.join(REPO, "nnet-asr_amd"))
    import tnet_amd  # noqa: F401  (maps torch's runtime first when torch is installed)
    from tnet_amd._lib import lib
    lib()
    seen = set()
    for line in open("/proc/self/maps"):
        p = line.split()[-1]
        if any(s in p for s in ("librccl", "libamdhip64", "libtnet_amd")):
            seen.add(os.path.realpath(p))
    return sorted(seen)


def kernels_of(path, tmp):
    fat = os.path.join(tmp, "fatbin.bin")
    co = os.path.join(tmp, "gfx950.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, fat], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    os.unlink(fat)
    os.unlink(co)
    out = []
    # each kernel's metadata is an indented YAML map starting at '- .agpr_count' / '.args'; scan by name
    for m in re.finditer(r"^\s+\.name:\s+(\S+)$", notes, re.M):
        name = m.group(1)
        if "Kernel" not in name or ("nccl" not in name.lower() and "rccl" not in name.lower()):
            continue
        # the block of this kernel: from the previous '  - ' item start to the next one
        start = notes.rfind("\n  - ", 0, m.start())
        end = notes.find("\n  - ", m.end())
        blk = notes[start:end if end > 0 else len(notes)]

        def field(key):
            f = re.search(r"^\s+\." + key + r":\s+(\S+)$", blk, re.M)
            return int(f.group(1)) if f else None
        out.append({"name": name, "lds_bytes": field("group_segment_fixed_size"), "vgpr": field("vgpr_count"),
                    "agpr": field("agpr_count"), "sgpr": field("sgpr_count"),
                    "max_flat_workgroup_size": field("max_flat_workgroup_size"),
                    "vgpr_spill": field("vgpr_spill_count"), "private_bytes": field("private_segment_fixed_size")})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--out")
    a = ap.parse_args()
    mapped = mapped_runtime()
    libs = a.libs or sorted({p for p in mapped if "librccl" in p} | {os.path.realpath("/opt/rocm/lib/librccl.so.1")})
    res = {"mapped_in_python_process": mapped, "libraries": {}}
    with tempfile.TemporaryDirectory() as tmp:
        for p in libs:
            res["libraries"][p] = kernels_of(p, tmp)
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
