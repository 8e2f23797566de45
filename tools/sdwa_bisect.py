"""Bisection of the round-3 k_emit codegen fault over its SDWA instructions
(profiles/r03_kemit_fault_study.md; ADVICE round 4, Makefile:35).

The failing build is round 4's study tree (study_wip/ = commit 71130cf +
profiles/r03_kemit_fault_wip.patch, not committed), built with the SDWA peephole
ON and -DSTUDY_DETRANK (walk order fixed).  This tool takes that build's device
assembly of entropy.hip and rewrites a chosen subset of k_emit's SDWA
instructions into their plain forms -- each sub-dword source extracted by a
v_bfe_{u32,i32} into a spare VGPR (v72/v73, above the kernel's 72), then the
VOP3 form of the same operation -- and relinks the library.  Every other
instruction, register and wait stays as the compiler emitted it, so a subset
whose rewrite makes the output exact holds the faulting instruction.

    python tools/sdwa_bisect.py list                 # k_emit's SDWA instructions, numbered
    python tools/sdwa_bisect.py build NAME SPEC      # SPEC: none | all | a:b[,c:d...] (indices)
    python tools/sdwa_bisect.py stage                # the python side the GPU run needs

Outputs go to sdwa_study/ (git-ignored, travels to the GPU box):
sdwa_study/libs/NAME/libdmmt_jpeg.so; scripts/gpu_sdwa_bisect.sh runs them.
"""
import os
import re
import shlex
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WIP = os.path.join(ROOT, "study_wip")
WPKG = os.path.join(WIP, "dmmt-jpeg-encoder_amd")
OUT = os.path.join(ROOT, "sdwa_study")
WORK = os.path.join(OUT, "work")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-result",
         "-DSTUDY_DETRANK"]
KEMIT = "_ZN4dmmt6k_emitEPKsS1_PKhPKjNS_4GeomEPjS7_S7_S7_S7_S7_"
SPARE = ("v72", "v73")
SEL = {"BYTE_0": (0, 8), "BYTE_1": (8, 8), "BYTE_2": (16, 8), "BYTE_3": (24, 8), "WORD_0": (0, 16),
       "WORD_1": (16, 16)}
SDWA_RE = re.compile(r"^(\s+)(v_\w+?)_sdwa\s+(.*?)\s+((?:dst_sel|src0_sel):.*)$")


def run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(f"failed: {' '.join(cmd)[:300]}\n{r.stderr[-2000:]}")
    return r


def device_asm():
    os.makedirs(WORK, exist_ok=True)
    s = os.path.join(WORK, "entropy_det.s")
    if not os.path.exists(s):
        run([HIPCC, *FLAGS, "--cuda-device-only", "-S", "csrc/entropy.hip", "-o", s], cwd=WPKG)
    return open(s).read().split("\n")


def kemit_range(lines):
    a = next(i for i, l in enumerate(lines) if l.startswith(KEMIT + ":"))
    b = next(i for i in range(a, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return a, b


def sdwa_lines(lines):
    a, b = kemit_range(lines)
    return [i for i in range(a, b) if SDWA_RE.match(lines[i])]


def rewrite(line):
    """The plain form of one SDWA instruction (dst_sel:DWORD, UNUSED_PAD only)."""
    ind, op, ops, mods = SDWA_RE.match(line).groups()
    mods = dict(m.split(":") for m in mods.split())
    assert mods.get("dst_sel", "DWORD") == "DWORD" and mods.get("dst_unused", "UNUSED_PAD") == "UNUSED_PAD", line
    assert not any(k not in ("dst_sel", "dst_unused", "src0_sel", "src1_sel") for k in mods), line
    parts = [p.strip() for p in ops.split(",")]
    dst, srcs = parts[0], parts[1:]
    out = []
    new = []
    for k, s in enumerate(srcs):
        sel = mods.get(f"src{k}_sel", "DWORD")
        sx = s.startswith("sext(")
        reg = s[5:-1] if sx else s
        assert not reg.startswith("-") and "|" not in reg, line
        if sel == "DWORD":
            assert not sx, line  # sext of a whole dword: not formed here
            new.append(reg)
            continue
        off, wid = SEL[sel]
        t = SPARE[k]
        out.append(f"{ind}v_bfe_{'i32' if sx else 'u32'} {t}, {reg}, {off}, {wid}")
        new.append(t)
    out.append(f"{ind}{op}_e64 {dst}, {', '.join(new)}")
    return out


def parse_spec(spec, n):
    if spec == "none":
        return set()
    if spec == "all":
        return set(range(n))
    sel = set()
    for part in spec.split(","):
        a, b = part.split(":")
        sel |= set(range(int(a), min(int(b), n)))
    return sel


def patched_asm(spec):
    lines = device_asm()
    idx = sdwa_lines(lines)
    chosen = parse_spec(spec, len(idx))
    rep = {idx[j]: rewrite(lines[idx[j]]) for j in chosen}
    a0, b0 = kemit_range(lines)
    assert not any(re.search(r"\bv7[2-9]\b|v\[7[0-9]:|v\[[0-9]+:7[2-9]\]", lines[i]) for i in range(a0, b0)), "spare used"
    out = []
    for i, l in enumerate(lines):
        out.extend(rep.get(i, [l]))
    if chosen:  # two spare VGPRs for k_emit: descriptor and metadata
        a, b = kemit_range(out)
        for i in range(a, b):  # (the kernel descriptor lies inside the function's range)
            out[i] = out[i].replace(".amdhsa_next_free_vgpr 72", ".amdhsa_next_free_vgpr 74")
            out[i] = out[i].replace(".amdhsa_accum_offset 72", ".amdhsa_accum_offset 76")
        nm = next(i for i, l in enumerate(out) if l.strip() == f".name:           {KEMIT}")
        vc = next(i for i in range(nm, len(out)) if out[i].strip().startswith(".vgpr_count:"))
        assert out[vc].strip() == ".vgpr_count:     72", out[vc]
        out[vc] = out[vc].replace("72", "74")
    return out, len(chosen), len(idx)


def build(name, spec):
    out, nsel, n = patched_asm(spec)
    d = os.path.join(WORK, name)
    os.makedirs(d, exist_ok=True)
    s = os.path.join(d, "entropy.s")
    open(s, "w").write("\n".join(out))
    llvm = "/opt/rocm/lib/llvm/bin"
    run([f"{llvm}/clang", "-x", "assembler", "--target=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", s, "-o",
         os.path.join(d, "dev.o")])
    run([f"{llvm}/lld", "-flavor", "gnu", "-m", "elf64_amdgpu", "--no-undefined", "-shared", "-o",
         os.path.join(d, "dev.out"), os.path.join(d, "dev.o")])
    run([f"{llvm}/clang-offload-bundler", "-type=o", "-bundle-align=4096",
         "-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950", "-input=/dev/null",
         f"-input={os.path.join(d, 'dev.out')}", f"-output={os.path.join(d, 'entropy.hipfb')}"])
    # the host half: the driver's own host command with this fat binary
    r = run([HIPCC, *FLAGS, "-c", "csrc/entropy.hip", "-o", os.path.join(d, "entropy.o"), "-###"], cwd=WPKG)
    host = [shlex.split(l) for l in r.stderr.split("\n") if l.startswith(" \"") and "-fcuda-include-gpubinary" in l]
    assert len(host) == 1
    cmd = host[0]
    cmd[cmd.index("-fcuda-include-gpubinary") + 1] = os.path.join(d, "entropy.hipfb")
    run(cmd, cwd=WPKG)
    objs = [os.path.join(d, "entropy.o")] + [os.path.join(WPKG, "build_det", f"{o}.o")
                                             for o in ("kernels", "ppm_device", "encoder", "tables", "ppm")]
    lib = os.path.join(OUT, "libs", name)
    os.makedirs(lib, exist_ok=True)
    run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(lib, "libdmmt_jpeg.so"), *objs,
         "-Wl,-soname,libdmmt_jpeg.so"])
    print(f"{name}: {nsel} of {n} SDWA instructions of k_emit rewritten -> {lib}")


def stage():
    """The study tree's python side (wrapper, oracle, determinism script) next to the libs."""
    for src, dst in (("dmmt-jpeg-encoder_amd/dmmt_jpeg.py", "dmmt-jpeg-encoder_amd/dmmt_jpeg.py"),
                     ("scripts/debug_determinism.py", "scripts/debug_determinism.py")):
        os.makedirs(os.path.dirname(os.path.join(OUT, dst)), exist_ok=True)
        shutil.copy(os.path.join(WIP, src), os.path.join(OUT, dst))
    if os.path.exists(os.path.join(OUT, "oracle")):
        shutil.rmtree(os.path.join(OUT, "oracle"))
    shutil.copytree(os.path.join(WIP, "oracle"), os.path.join(OUT, "oracle"),
                    ignore=shutil.ignore_patterns("__pycache__"))
    # the shipped failing build and its no-SDWA control, as built in round 4
    for v in ("lib_det", "lib_detnosdwa"):
        os.makedirs(os.path.join(OUT, "libs", v), exist_ok=True)
        shutil.copy(os.path.join(WPKG, v, "libdmmt_jpeg.so"), os.path.join(OUT, "libs", v, "libdmmt_jpeg.so"))


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "list":
        lines = device_asm()
        for j, i in enumerate(sdwa_lines(lines)):
            print(j, i + 1, lines[i].strip())
    elif cmd == "build":
        build(sys.argv[2], sys.argv[3])
    elif cmd == "stage":
        stage()
    else:
        sys.exit(__doc__)
