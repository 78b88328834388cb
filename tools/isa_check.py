"""Static checks of the gfx950 device assembly of the library's HIP sources.

  python tools/isa_check.py [source.hip ...]      (default: every csrc/*.hip)

Compiles each source with the library's flags to device assembly (hipcc --cuda-device-only -S) and reports, per
kernel:
  * waterfall loops around buffer loads / stores -- a buffer resource built from a value the compiler cannot
    prove wave-uniform (e.g. a per-problem offset read from device memory) wraps every buffer access in a
    readfirstlane / compare / exec loop, and the loop-carried destination adds a vmcnt(0) per access;
  * scratch (private memory) instructions -- spills or a kernel-argument copy that lives in memory.
Exit status 1 if any kernel has a waterfall loop.
"""
import concurrent.futures as cf
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "collaborative_nonstationary_multivariate_gaussian_process_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S"]


def scan(asm_text):
    lines = asm_text.split("\n")
    name = None
    out = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            name = m.group(1)
            out.setdefault(name, {"waterfall": 0, "scratch": 0})
        if name is None:
            continue
        if "s_xor_b64 exec, exec" in l and i + 1 < len(lines) and "s_cbranch_execnz" in lines[i + 1]:
            blk = "\n".join(lines[max(0, i - 12):i])
            if "v_readfirstlane" in blk and "buffer_" in blk:
                out[name]["waterfall"] += 1
        s = l.strip()
        if s.startswith("scratch_"):
            out[name]["scratch"] += 1
    return out


def check(src):
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        r = subprocess.run([HIPCC] + FLAGS + [src, "-o", asm], capture_output=True, text=True, cwd=os.path.dirname(src))
        if r.returncode != 0:
            raise RuntimeError(f"{src}: hipcc failed\n{r.stderr[-2000:]}")
        return scan(open(asm).read())


def main(srcs=None):
    srcs = srcs or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    bad = {}
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        for src, res in zip(srcs, ex.map(check, srcs)):
            for k, v in res.items():
                if v["waterfall"] or v["scratch"]:
                    print(json.dumps({"source": os.path.basename(src), "kernel": k[:90], **v}))
                if v["waterfall"]:
                    bad[k] = v
    return bad


if __name__ == "__main__":
    sys.exit(1 if main([os.path.abspath(p) for p in sys.argv[1:]]) else 0)
