"""Scan gfx950 device code for a VALU-written SGPR read by a VMEM instruction fewer than 5 wait states later.

CDNA3/4 needs five wait states between a VALU op that writes an SGPR (v_readfirstlane, v_readlane, v_cmp into an SGPR
pair) and a VMEM instruction that reads it as its buffer resource or soffset. The compiler pads its own VMEM
instructions; it cannot see into inline asm, so a hand-written `buffer_load ... lds` / `buffer_store` whose resource
the compiler materialised (or reloaded from an SGPR spill lane) right in front of it reads a stale SGPR -- the
illegal-address faults of round 4 in gemm4w's direct epilogue (csrc/kernels/gemm4w.h, store16_padded).

  python tools/sgpr_hazard.py build/kernels/gemm4w_01.o      # object / shared library: gfx950 bundle disassembled
  python tools/sgpr_hazard.py /tmp/k.s                       # or assembly from tools/asm_kernel.sh

Prints each hazard and a final `hazards N`; exit status 1 when N > 0.
"""
import os
import re
import subprocess
import sys
import tempfile

WAIT = 5
LLVM = "/opt/rocm/lib/llvm/bin"


# SALU / control ops that read SGPRs but write none (their first operand is a source): they do not end a hazard
NO_SDST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_setreg", "s_setprio", "s_sleep", "s_sendmsg", "s_trap",
           "s_waitcnt", "s_barrier", "s_nop", "s_endpgm", "s_set_gpr_idx", "s_dcache", "s_icache", "s_incperflevel",
           "s_decperflevel", "s_ttracedata", "s_setkill")
M0 = -1   # m0 (the LDS-DMA destination base) as a pseudo-SGPR


def sgprs(tok):
    tok = tok.strip()
    if tok == "m0":
        return {M0}
    m = re.match(r"s\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def disassemble(path):
    """device assembly text of the gfx950 code object bundled in an object file / shared library"""
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "co")
        r = subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", path,
                            os.path.join(td, "x")], capture_output=True)
        if r.returncode != 0:   # host-only object (no device code)
            return ""
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                              capture_output=True, text=True).stdout


def scan(text, name="<asm>"):
    """list of hazard descriptions in one assembly / disassembly text"""
    func = "?"
    hist = []   # (SGPRs written by a VALU op, wait states since its issue, source text)
    out = []
    for ln, raw in enumerate(text.splitlines(), 1):
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", raw) or re.match(r"^([_A-Za-z][\w.$]*):", raw)
        if m:
            if m.group(1).startswith("_Z"):
                func, hist = m.group(1), []   # a new function (labels inside one keep the fall-through history)
            continue
        line = raw.split(";")[0].split("//")[0].strip()
        if not line or line.startswith("."):
            continue
        op = line.split()[0]
        args = line[len(op):].split(",")
        ws = int(args[0], 0) + 1 if op == "s_nop" else 1
        lds = op.startswith("buffer_") and re.search(r"\slds\b", line) is not None
        if op.startswith("buffer_") and (len(args) >= 4 or (lds and len(args) >= 3)):
            # LDS-DMA form `buffer_load_dwordx4 vaddr, srsrc, soffset offen lds` (no VGPR destination; reads m0)
            # vs `buffer_op vdata, vaddr, srsrc, soffset ...`
            if lds and len(args) == 3:
                reads = sgprs(args[1]) | sgprs(args[2].split()[0]) | {M0}
            else:
                reads = sgprs(args[2]) | sgprs(args[3].split()[0]) | ({M0} if lds else set())
            for w, age, src in hist:
                if w & reads and age < WAIT:
                    out.append(f"{name}:{ln}: {line}  <- {src} ({age} wait states) in {func[:70]}")
        if op.startswith("v_") and not op.startswith("v_mfma") and args:
            w = sgprs(args[0])
            if w:
                hist.append((w, -ws, f"{op} {args[0].strip()}"))
        if op.startswith("s_") and args and not op.startswith(NO_SDST):
            w = sgprs(args[0])   # an SALU rewrite of the SGPR ends its hazard (only ops with an SGPR destination)
            hist = [(h - w, a, s) for h, a, s in hist if h - w]
        hist = [(h, a + ws, s) for h, a, s in hist if a + ws < 16]
    return out


def main(paths):
    n = 0
    for p in paths:
        text = open(p).read() if p.endswith(".s") else disassemble(p)
        for h in scan(text, p):
            print(h)
            n += 1
    print("hazards", n)
    return 1 if n else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
