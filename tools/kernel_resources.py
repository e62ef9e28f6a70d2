"""Per-kernel resources of the gfx950 code object inside a built library: VGPRs, AGPRs, SGPRs, LDS and
the private segment (scratch) of every kernel, from the code object's metadata notes.

    python tools/kernel_resources.py [lib.so] [--grep k_step] [--json out.json]

(llvm-objcopy dumps .hip_fatbin, clang-offload-bundler unbundles the gfx950 object, llvm-readelf
prints its AMDGPU metadata; no GPU needed.)
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_object(lib, tmp):
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(tmp, "junk")],
                   check=True)
    co = os.path.join(tmp, "gfx950.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
    return co


def kernels(co):
    text = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True, check=True).stdout
    out = []
    for block in re.split(r"\n\s+- \.agpr_count:", text)[1:]:
        block = ".agpr_count:" + block

        def field(name):
            m = re.search(r"\." + name + r":\s+(\S+)", block)
            return m.group(1) if m else None

        out.append({"name": field("name"), "vgpr": int(field("vgpr_count") or 0), "agpr": int(field("agpr_count") or 0),
                    "sgpr": int(field("sgpr_count") or 0), "lds": int(field("group_segment_fixed_size") or 0),
                    "scratch": int(field("private_segment_fixed_size") or 0)})
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "rllib-warehouse_amd", "warehouse", "_lib",
                                                           "libwarehouse_amd.so"))
    ap.add_argument("--grep", default="")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as tmp:
        ks = kernels(code_object(a.lib, tmp))
    for k, d in zip(ks, demangle([k["name"] for k in ks])):
        k["demangled"] = d
    ks = [k for k in ks if a.grep in k["demangled"]]
    for k in sorted(ks, key=lambda k: k["demangled"]):
        print(f"{k['vgpr']:4d} v {k['agpr']:4d} a {k['sgpr']:3d} s {k['lds']:7d} lds {k['scratch']:5d} scratch  {k['demangled'][:150]}")
    if a.json:
        json.dump(ks, open(a.json, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
