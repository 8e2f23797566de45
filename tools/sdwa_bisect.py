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
    python tools/sdwa_bisect.py build NAME SPEC [VGPRS [LDS [INIT]]]
        SPEC: none | all | a:b[,c:d...] (indices), k:... in place (no spare
        registers); VGPRS / LDS: k_emit's register count / LDS bytes in its
        descriptor (no code change; '-' keeps it); INIT: VGPRs zeroed at the
        kernel's entry, e.g. 1-71 or 1-18,37-54 (v0 holds the work-item ids)
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


def rewrite(line, keep=False):
    """The plain form of one SDWA instruction (dst_sel:DWORD, UNUSED_PAD only).
    keep: no spare registers -- the destination VGPR takes the extracted source
    (None when it cannot: a compare, or a destination that is also a source)."""
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
        if keep:
            others = [x[5:-1] if x.startswith("sext(") else x for j, x in enumerate(srcs) if j != k]
            if not re.fullmatch(r"v\d+", dst) or dst in others or sum(mods.get(f"src{j}_sel", "DWORD") != "DWORD"
                                                             for j in range(len(srcs))) != 1:
                return None
            t = dst
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


def parse_regs(init):
    regs = []
    for part in init.split(","):
        a, _, b = part.partition("-")
        regs += list(range(int(a), int(b or a) + 1))
    assert all(1 <= r for r in regs)
    return regs


def patched_asm(spec, vgprs=None, lds=None, init=None):
    lines = device_asm()
    ren = os.environ.get("SDWA_RENAME")  # "71:79": k_emit's v71 renamed (a register-placement control)
    if ren:
        f, t = ren.split(":")
        a0, b0 = kemit_range(lines)
        assert not any(re.search(rf"\bv{t}\b|v\[\d+:\d+\]", lines[i]) and re.search(rf"v\[\d+:{f}\]|v\[{f}:", lines[i])
                       for i in range(a0, b0)), "renamed register inside a tuple"
        code_end = next(i for i in range(a0, b0) if lines[i].strip().startswith(".section"))
        lines = [re.sub(rf"\bv{f}\b", f"v{t}", l) if a0 <= i < code_end else l for i, l in enumerate(lines)]
    sub = os.environ.get("SDWA_SUB")  # "old=>new": one exact k_emit instruction replaced (\n: several)
    if sub:
        f, t = sub.split("=>")
        a0, b0 = kemit_range(lines)
        hits = [i for i in range(a0, b0) if lines[i].strip() == f]
        assert len(hits) == 1, (f, len(hits))
        lines[hits[0]] = "\n".join("\t" + x for x in t.split("\\n"))
        lines = "\n".join(lines).split("\n")
    idx = sdwa_lines(lines)
    keep = spec.startswith("k:")  # rewrite in place, no spare registers (occupancy unchanged)
    chosen = parse_spec(spec[2:] if keep else spec, len(idx))
    rep = {idx[j]: rewrite(lines[idx[j]], keep) for j in chosen}
    rep = {i: r for i, r in rep.items() if r is not None}
    chosen = rep if keep else chosen
    a0, b0 = kemit_range(lines)
    assert keep or not chosen or not any(re.search(r"\bv7[2-9]\b|v\[7[0-9]:|v\[[0-9]+:7[2-9]\]", lines[i])
                                         for i in range(a0, b0)), "spare used"
    out = []
    for i, l in enumerate(lines):
        out.extend(rep.get(i, [l]))
    if chosen and vgprs is None and not keep:
        vgprs = 74  # two spare VGPRs for k_emit
    if init:  # entry: zero the chosen VGPRs (their contents are otherwise what the last wave left)
        e = next(i for i, l in enumerate(out) if l.startswith(KEMIT + ":")) + 1
        out[e:e] = [f"\tv_mov_b32_e32 v{r}, 0" for r in parse_regs(init)]
    a, b = kemit_range(out)
    nm = next(i for i, l in enumerate(out) if l.strip() == f".name:           {KEMIT}")
    if vgprs is not None:  # descriptor and metadata
        for i in range(a, b):  # (the kernel descriptor lies inside the function's range)
            out[i] = out[i].replace(".amdhsa_next_free_vgpr 72", f".amdhsa_next_free_vgpr {vgprs}")
            out[i] = out[i].replace(".amdhsa_accum_offset 72", f".amdhsa_accum_offset {(vgprs + 3) & ~3}")
        vc = next(i for i in range(nm, len(out)) if out[i].strip().startswith(".vgpr_count:"))
        assert out[vc].strip() == ".vgpr_count:     72", out[vc]
        out[vc] = out[vc].replace("72", str(vgprs))
    if lds is not None:
        for i in range(a, b):
            out[i] = out[i].replace(".amdhsa_group_segment_fixed_size 22880", f".amdhsa_group_segment_fixed_size {lds}")
        # (the metadata entry of k_emit precedes its .name line)
        gs = max(i for i in range(nm) if out[i].strip().startswith(".group_segment_fixed_size:"))
        assert out[gs].strip() == ".group_segment_fixed_size: 22880", out[gs]
        out[gs] = out[gs].replace("22880", str(lds))
    return out, len(chosen), len(idx)


def build(name, spec, vgprs=None, lds=None, init=None):
    out, nsel, n = patched_asm(spec, vgprs, lds, init)
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
    print(f"{name}: {nsel} of {n} SDWA instructions of k_emit rewritten, vgprs {vgprs}, lds {lds}, init {init} -> {lib}")


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
        opt = [int(x) if x != "-" else None for x in sys.argv[4:6]]
        opt += [None] * (2 - len(opt))
        build(sys.argv[2], sys.argv[3], *opt, sys.argv[6] if len(sys.argv) > 6 else None)
    elif cmd == "stage":
        stage()
    else:
        sys.exit(__doc__)
