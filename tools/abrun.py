"""Same-box A/B runs of library variants, reproducible from the tree.

One spec names every library of an experiment and how it is built, so each result file says which
command rebuilds what it measured:

    python tools/abrun.py build SPEC.json        # here (CPU): build every variant into build_ab/
    python tools/abrun.py run SPEC.json          # GPU box: interleaved rounds -> gpurun_out/<out>
    python tools/abrun.py show SPEC.json         # the recipes, as written into the result header

SPEC.json:
    {"out": "r05_prologue_ab.txt",                    # result file (gpurun_out/, then copied to profiles/)
     "rounds": 2,
     "variants": [
        {"name": "tree"},                             # the production library of this tree
        {"name": "noprog", "flags": "-DWH_X"},        # this tree's sources with -D flags (build_variant.sh)
        {"name": "r04", "rev": "f6d71ed"},            # the library at a git revision (its own Makefile)
        {"name": "r04x", "rev": "f6d71ed", "flags": "-DWH_Y"},
        {"name": "l16", "flags": "-DWH_ONLY_LARGE16", "commands": ["..."]},   # own commands
        {"name": "ilp", "flags": "-DWH_ONLY_MEDIUM8", "sched": "-mllvm -amdgpu-sched-strategy=max-ilp"},   # scheduler
        {"name": "tree_x", "lib": "tree", "env": {"WH_SAMPLER_UNFUSED": "1"}}],   # same library, env
     "commands": ["python tools/step_probe.py --steps 200 --launches 6",
                  "python tools/step_probe.py --variant large --agents 16 --steps 20 --launches 8"],
     "timeout": 180}

`run` loads each variant through WAREHOUSE_AMD_LIB (WAREHOUSE_AMD_AB=1 lets a library of another
revision, which may lack newer entry points, load), alternates variants within every round so clock
drift hits all of them, puts every command under its own `timeout -k 10`, stops at the first failure,
and writes a header with each variant's recipe and its wh_version() string before the results.
"""
from __future__ import annotations

import json
import os
import shlex
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rllib-warehouse_amd", "csrc")
PROD = os.path.join(ROOT, "rllib-warehouse_amd", "warehouse", "_lib", "libwarehouse_amd.so")


def lib_path(v):
    """A variant's library; "lib" names another variant's (the same library under other env settings)."""
    name = v.get("lib", v["name"])
    return PROD if name == "tree" else os.path.join(ROOT, "build_ab", f"{name}.so")


def recipe(v):
    """The command that rebuilds variant v's library from this repository."""
    if "lib" in v:
        return f"the library of variant {v['lib']}, run with {v.get('env', {})}"
    if v["name"] == "tree":
        return "make -C rllib-warehouse_amd/csrc (the production library of this tree)"
    if "rev" in v:
        return (f"git archive {v['rev']} rllib-warehouse_amd/csrc include | tar -x -C build/rev_{v['name']} && "
                f"make -C build/rev_{v['name']}/rllib-warehouse_amd/csrc OUT=$PWD/{os.path.relpath(lib_path(v), ROOT)} "
                + (f"EXTRA='{v['flags']}'" if v.get("flags") else ""))
    pre = f"SCHED='{v['sched']}' " if v.get("sched") else ""
    return f"{pre}bash tools/build_variant.sh {v['name']} {v.get('flags', '')}".strip()


def build(spec):
    for v in spec["variants"]:
        if "lib" in v:
            continue
        if v["name"] == "tree":
            cmd = ["make", "-s", "-C", CSRC, "-j2"]
            subprocess.run(cmd, check=True)
            continue
        os.makedirs(os.path.join(ROOT, "build_ab"), exist_ok=True)
        if "rev" in v:
            dst = os.path.join(ROOT, "build", f"rev_{v['name']}")
            shutil.rmtree(dst, ignore_errors=True)   # objects of an earlier revision would look newer
            os.makedirs(dst, exist_ok=True)
            arch = subprocess.run(["git", "-C", ROOT, "archive", v["rev"], "rllib-warehouse_amd/csrc", "include"],
                                  check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", dst], input=arch, check=True)
            cmd = ["make", "-s", "-C", os.path.join(dst, "rllib-warehouse_amd", "csrc"), "-j2", f"OUT={lib_path(v)}",
                   f"OBJDIR={os.path.join(dst, 'obj')}"]
            if v.get("flags"):
                cmd.append(f"EXTRA={v['flags']}")
            subprocess.run(cmd, check=True)
        else:
            env = dict(os.environ, SCHED=v["sched"]) if v.get("sched") else None   # the step object's scheduler flags
            subprocess.run(["bash", os.path.join(ROOT, "tools", "build_variant.sh"), v["name"]]
                           + shlex.split(v.get("flags", "")), check=True, env=env)
        print(f"built {v['name']}: {lib_path(v)}", flush=True)


def version_of(path):
    code = ("import ctypes,sys; L=ctypes.CDLL(sys.argv[1]); L.wh_version.restype=ctypes.c_char_p; "
            "print(L.wh_version().decode())")
    r = subprocess.run([sys.executable, "-c", code, path], capture_output=True, text=True, timeout=60)
    return r.stdout.strip() or f"(unreadable: {r.stderr.strip()[-200:]})"


def header(spec):
    lines = [f"# tools/abrun.py run {spec.get('_path', 'SPEC')} -- {spec.get('note', '')}".rstrip(" -")]
    for v in spec["variants"]:
        lines.append(f"# variant {v['name']}: {recipe(v)}")
    return lines


def run(spec):
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, spec["out"])
    tmo = int(spec.get("timeout", 180))
    with open(out, "w") as f:
        for ln in header(spec):
            f.write(ln + "\n")
        for v in spec["variants"]:
            f.write(f"# variant {v['name']} wh_version: {version_of(lib_path(v))}\n")
    for rnd in range(int(spec.get("rounds", 2))):
        for v in spec["variants"]:
            env = dict(os.environ, WAREHOUSE_AMD_LIB=lib_path(v), WAREHOUSE_AMD_AB="1", **v.get("env", {}))
            for cmd in (v["commands"] if "commands" in v else spec["commands"]):
                with open(out, "a") as f:
                    f.write(f"lib={v['name']} round={rnd + 1} cmd={cmd}\n")
                    f.flush()
                    r = subprocess.run(["timeout", "-k", "10", str(tmo)] + shlex.split(cmd), cwd=ROOT, env=env,
                                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
                    f.write("".join(ln + "\n" for ln in r.stdout.splitlines() if "amdgpu.ids" not in ln))
                if r.returncode:
                    print(f"abrun: {v['name']} `{cmd}` exited {r.returncode}; stopping", flush=True)
                    return r.returncode
            print(f"abrun: round {rnd + 1} {v['name']} done", flush=True)
    print(open(out).read())
    return 0


def main():
    if len(sys.argv) != 3 or sys.argv[1] not in ("build", "run", "show"):
        print(__doc__)
        return 2
    spec = json.load(open(sys.argv[2]))
    spec["_path"] = os.path.relpath(os.path.abspath(sys.argv[2]), ROOT)
    if sys.argv[1] == "build":
        build(spec)
    elif sys.argv[1] == "run":
        return run(spec)
    else:
        print("\n".join(header(spec)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
