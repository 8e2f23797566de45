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

    python tools/last_vgpr_check.py [LIB.so]     # exit 1 when any is found

The device code objects are read from the library's .hip_fatbin section (clang
offload bundles); llvm-objdump / llvm-readelf from /opt/rocm disassemble them.
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
GRANULE = 8  # gfx950 wave64 VGPR allocation granule
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


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


def code_objects(lib):
    """Every gfx950 code object of the library's fat binary."""
    fb = elf_section(lib, ".hip_fatbin")
    assert fb is not None, f"{lib}: no .hip_fatbin section"
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
    assert out, f"{lib}: no gfx950 code object (a compressed bundle is not handled)"
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
    kern = None
    for line in dis.split("\n"):
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            kern = m.group(1)
            continue
        if kern not in counts:
            continue
        ins = line.strip().split(" //")[0]
        mn = ins.split(" ")[0] if ins else ""
        if not mn.startswith("v_") or not re.search(r"_(b|u|i|f)64", mn):
            continue
        last = (counts[kern] + GRANULE - 1) // GRANULE * GRANULE - 1
        ops = ins[len(mn):]
        if re.search(rf"(?<![\[:\w])v{last}\b(?!:)", ops):
            hits.append((kern, counts[kern], last, ins))
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
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "dmmt-jpeg-encoder_amd", "lib",
                                                                        "libdmmt_jpeg.so")))
