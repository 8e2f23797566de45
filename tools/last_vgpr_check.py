"""Check a built library's gfx950 kernels for the round-3 k_emit fault pattern.

The fault (profiles/r03_kemit_fault_study.md, round 5): a
`v_lshlrev_b64 v[a:a+1], vS, v[b:b+1]` whose 32-bit shift amount vS is the LAST
VGPR of the wave's allocation computed different bits from run to run on
MI355X.  The same machine code with the amount in any other register, or with
the allocation grown past it, was exact.  In isolation
(tools/last_vgpr_probe.hip) the three 64-bit shifts take their amount from v0 in
~0.017 % of executions when it sits in the last VGPR; nine other instructions
reading that register were exact.  This tool is wider on purpose: it lists every
64-bit VALU operation (mnemonic with b64/u64/i64/f64) that reads a single VGPR
which is the last one of its kernel's allocation (vgpr_count rounded up to the
granule of 8).

    python tools/last_vgpr_check.py [--llvm DIR] [LIB.so]     # exit 1 when any is found

A symbol that is not a kernel (a device function the compiler did not inline)
runs with its caller's allocation: its 64-bit operations are checked against
the last VGPR of every kernel of its code object.

The device code objects are read from the library's .hip_fatbin section: plain
clang offload bundles are parsed here, compressed ones (CCOB, --offload-compress)
are unpacked with clang-offload-bundler.  llvm-objdump / llvm-readelf /
clang-offload-bundler come from --llvm DIR, else $LLVM_BIN, else
$ROCM_PATH/lib/llvm/bin (ROCM_PATH default /opt/rocm); the Makefile passes the
directory next to the hipcc it builds with.

Why this pattern: LLVM carries a hazard workaround for the same shape on gfx90a
(GCNHazardRecognizer::fixShift64HighRegBug -- a 64-bit shift whose amount sits in
the highest VGPR of an allocation block -- gated by GCNSubtarget::
hasShift64HighRegBug(), which is true for gfx90a only, so nothing is done for
gfx940 and later).  When the compiler enables it for gfx950 this guard can go.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = os.environ.get("LLVM_BIN") or os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")
GRANULE = 8  # gfx950 wave64 VGPR allocation granule
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
CCOB_MAGIC = b"CCOB"  # a compressed offload bundle


def elf_section(path, name):
    data = open(path, "rb").read()
    assert data[:4] == b"\x7fELF" and data[4] == 2, "ELF64 expected"
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    for s in secs:
        nm = data[stro + s[0]:data.index(b"\0", stro + s[0])].decode()
        if nm == name:
            return data[s[4]:s[4] + s[5]]
    return None


def compressed_code_objects(fb):
    """gfx950 code objects of the compressed bundles (CCOB) in a fat binary, each
    unpacked by clang-offload-bundler (the bundles lie back to back, padded)"""
    starts = []
    pos = fb.find(CCOB_MAGIC)
    while pos >= 0:
        starts.append(pos)
        pos = fb.find(CCOB_MAGIC, pos + 4)
    out = []
    with tempfile.TemporaryDirectory() as d:
        for i, a in enumerate(starts):
            b = starts[i + 1] if i + 1 < len(starts) else len(fb)
            src = os.path.join(d, f"b{i}.bin")
            with open(src, "wb") as f:
                f.write(fb[a:b])
            bundler = os.path.join(LLVM, "clang-offload-bundler")
            tgts = subprocess.run([bundler, "--type=o", f"--input={src}", "--list"], capture_output=True, text=True,
                                  check=True).stdout.split()
            for t in tgts:
                if "gfx950" not in t:
                    continue
                dst = os.path.join(d, f"b{i}.co")
                subprocess.run([bundler, "--type=o", f"--input={src}", "--unbundle", f"--targets={t}",
                                f"--output={dst}"], check=True)
                out.append(open(dst, "rb").read())
    return out


def code_objects(lib):
    """Every gfx950 code object of the library's fat binary."""
    fb = elf_section(lib, ".hip_fatbin")
    assert fb is not None, f"{lib}: no .hip_fatbin section"
    if fb.find(BUNDLE_MAGIC) < 0 and fb.find(CCOB_MAGIC) >= 0:
        out = compressed_code_objects(fb)
        assert out, f"{lib}: no gfx950 code object in its compressed bundles"
        return out
    out = []
    pos = fb.find(BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", fb, p)
            tid = fb[p + 24:p + 24 + idlen].decode()
            p += 24 + idlen
            if "gfx950" in tid and size:
                out.append(fb[pos + off:pos + off + size])
        pos = fb.find(BUNDLE_MAGIC, pos + 1)
    assert out, f"{lib}: no gfx950 code object"
    return out


def vgpr_counts(co_path):
    """kernel symbol -> .vgpr_count, from the code object's metadata note (one
    "- .agpr_count: ..." block per kernel, its keys in any order)"""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co_path], capture_output=True, text=True,
                           check=True).stdout
    counts = {}
    for b in re.split(r"\n\s+- \.", notes):
        n = re.search(r"\.name:\s+(\S+)", b)
        v = re.search(r"\.vgpr_count:\s+(\d+)", b)
        if n and v:
            counts[n.group(1)] = int(v.group(1))
    return counts


def check_object(co):
    with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
        f.write(co)
        path = f.name
    try:
        counts = vgpr_counts(path)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", path], capture_output=True,
                             text=True, check=True).stdout
    finally:
        os.unlink(path)
    hits = []
    sym = None
    lasts = {(c + GRANULE - 1) // GRANULE * GRANULE - 1: c for c in counts.values()}  # for non-kernel symbols
    for line in dis.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            sym = m.group(1)
            continue
        if sym is None or sym.startswith("__"):  # (none yet, or a runtime-internal symbol)
            continue
        ins = line.strip().split(" //")[0]
        mn = ins.split(" ")[0] if ins else ""
        if not mn.startswith("v_") or not re.search(r"_(b|u|i|f)64", mn):
            continue
        ops = ins[len(mn):]
        if sym in counts:  # a kernel: its own allocation
            cands = {(counts[sym] + GRANULE - 1) // GRANULE * GRANULE - 1: counts[sym]}
        else:  # a device function: any caller's allocation
            cands = lasts
        for last, cnt in cands.items():
            if re.search(rf"(?<![\[:\w])v{last}\b(?!:)", ops):
                hits.append((sym if sym in counts else f"{sym} (device function)", cnt, last, ins))
    return hits, len(counts)


def main(lib):
    hits, nk = [], 0
    for co in code_objects(lib):
        h, n = check_object(co)
        hits += h
        nk += n
    for kern, cnt, last, ins in hits:
        print(f"{kern}: vgpr_count {cnt}, last allocated v{last}: {ins}")
    print(f"{nk} kernels checked, {len(hits)} 64-bit operations reading the last allocated VGPR")
    return 1 if hits else 0


if __name__ == "__main__":
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    argv = sys.argv[1:]
    if len(argv) >= 2 and argv[0] == "--llvm":
        LLVM = argv[1]
        argv = argv[2:]
    sys.exit(main(argv[0] if argv else os.path.join(here, "dmmt-jpeg-encoder_amd", "lib", "libdmmt_jpeg.so")))
