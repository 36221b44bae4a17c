"""The exact search kernel keeps its accumulators in AGPRs outside the compiler's register model
(crimp_amd/csrc/search_exact.h, ex_mfma): any AGPR access hipcc generates itself -- a VGPR spilled to an AGPR under
register pressure, which resource-usage reports do not count as a spill -- would overwrite them. Compiles the
device code to assembly and lists such accesses (outside inline-asm blocks) in the k_search_exact kernels.
usage: python tools/agpr_check.py [-DNAME=VALUE ...]   (exit status 1 if any)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "crimp_amd", "csrc")


def compile_cmd(out, defines=(), asm=True):
    """hipcc command building the library's gfx950 device code with ``defines``: assembly (asm) or a bare code object"""
    return ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-w", "--cuda-device-only"] + (
        ["-S"] if asm else ["--no-gpu-bundle-output", "-c"]) + list(defines) + ["-o", out, "crimp_hip.hip"]


def accesses(text, kernel="k_search_exact"):
    """{kernel symbol: [compiler-generated lines naming an AGPR]} of a device assembly listing."""
    found = {}
    for m in re.finditer(r"^(_Z\w*%s\w*):" % kernel, text, re.M):
        name = m.group(1)
        body = text[m.end():text.find(".Lfunc_end", m.end())]
        inasm, bad = False, []
        for line in body.splitlines():
            if "ASMSTART" in line:
                inasm = True
            elif "ASMEND" in line:
                inasm = False
            elif not inasm and re.search(r"\ba\d+\b|\ba\[\d+", line.split(";")[0]):
                bad.append(line.strip())
        found[name] = bad
    return found


def compiler_agpr_accesses(kernel="k_search_exact", defines=(), asm_path=None):
    """{kernel symbol: [compiler-generated lines naming an AGPR]} of the device code built with ``defines``
    (e.g. ("-DCRIMP_EX_AGPR_CLOBBERS=0", "-DCRIMP_EX_OPEN=0"): round 3's faulting build), or of an
    already built listing ``asm_path``."""
    if asm_path is not None:
        return accesses(open(asm_path).read(), kernel)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run(compile_cmd(out, defines), cwd=SRC, check=True, capture_output=True)
        return accesses(open(out).read(), kernel)


if __name__ == "__main__":
    res = compiler_agpr_accesses(defines=tuple(sys.argv[1:]))
    n = 0
    for name, bad in res.items():
        print("%s: %d compiler AGPR accesses %s" % (name, len(bad), bad[:4]))
        n += len(bad)
    sys.exit(1 if n or not res else 0)
