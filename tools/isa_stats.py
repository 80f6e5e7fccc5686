"""Per-kernel ISA statistics of built objects (measurement tooling, not product).

usage: python tools/isa_stats.py [FILE.o|FILE.so ...] [--filter SUBSTR] [--dump DIR]
Default: every object under optiland_pr_amd/lib/obj/. For each kernel prints the
instruction count, VGPR / AGPR / SGPR counts and scratch bytes (from the code object's
metadata notes), and with --dump writes the disassembly per object.
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def code_objects(path, tmp):
    fb = os.path.join(tmp, os.path.basename(path) + ".fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, path],
                   check=True, capture_output=True)
    co = os.path.join(tmp, os.path.basename(path) + ".co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", "--input=" + fb,
                    "--output=" + co, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"],
                   check=True, capture_output=True)
    return co


def stats(co):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                         capture_output=True, text=True).stdout
    counts, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1)
            counts[cur] = 0
        elif cur and line.strip() and not line.strip().startswith(";"):
            counts[cur] += 1
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                           text=True).stdout
    meta, name = {}, None
    for line in notes.splitlines():
        t = line.strip()
        m = re.match(r"\.name:\s+(\S+)", t)
        if m:
            name = m.group(1)
            meta[name] = {}
        for key in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size",
                    "vgpr_spill_count"):
            m = re.match(r"\." + key + r":\s+(\d+)", t)
            if m and name:
                meta[name][key] = int(m.group(1))
    return dis, counts, meta


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    if filt in args:
        args.remove(filt)
    if dump in args:
        args.remove(dump)
    files = args or sorted(glob.glob(os.path.join(REPO, "optiland_pr_amd/lib/obj/*.o")))
    with tempfile.TemporaryDirectory() as tmp:
        for f in files:
            try:
                co = code_objects(f, tmp)
            except subprocess.CalledProcessError:
                continue  # no device code in this object
            dis, counts, meta = stats(co)
            if dump:
                os.makedirs(dump, exist_ok=True)
                with open(os.path.join(dump, os.path.basename(f) + ".s"), "w") as fh:
                    fh.write(dis)
            for k, n in sorted(counts.items()):
                if "kernel" not in k or filt not in k:
                    continue
                md = meta.get(k, {})
                print(f"{os.path.basename(f):22s} {k[:70]:70s} insts={n:6d} "
                      f"vgpr={md.get('vgpr_count')} agpr={md.get('agpr_count')} "
                      f"sgpr={md.get('sgpr_count')} scratch={md.get('private_segment_fixed_size')}")


if __name__ == "__main__":
    main()
