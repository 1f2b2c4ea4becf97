#!/usr/bin/env python3
"""Dump the hipRTC step kernel of a bench config (no GPU needed): generated source, code object,
disassembly and resource usage, for instruction counts and register pressure.

    python tools/jit_dump.py C4 [OUTDIR] [--flags F]
"""
import ctypes
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "marl-for-im_amd")]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flags = 0
    if "--flags" in sys.argv:
        flags = int(sys.argv[sys.argv.index("--flags") + 1], 0)
        args = [a for a in args if a != sys.argv[sys.argv.index("--flags") + 1]]
    cname = args[0] if args else "C2"
    out = os.path.abspath(args[1] if len(args) > 1 else "/tmp/jit_dump_" + cname)
    os.makedirs(out, exist_ok=True)
    for f in glob.glob(os.path.join(out, "imenv_jit_*")):
        os.remove(f)
    os.environ["IMENV_JIT_DUMP"] = out
    import bench
    from imenv import _native, build_spec
    kind, cfg = bench.CONFIGS[cname][:2]
    spec = build_spec(kind, cfg).to_c()
    lib = _native.load()
    log = ctypes.create_string_buffer(1 << 16)
    rc = lib.imenv_jit_check(ctypes.byref(spec), b"gfx950", flags, log, len(log))
    if rc:
        raise SystemExit(log.value.decode())
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    for co in glob.glob(os.path.join(out, "imenv_jit_*.co")):
        dis = co[:-3] + ".s"
        with open(dis, "w") as f:
            subprocess.check_call([objdump, "-d", "--mcpu=gfx950", co], stdout=f)
        text = open(dis).read().splitlines()
        ins = [l.split()[0] for l in text if l.startswith("\t") or l.startswith("  ")]
        ins = [l.strip().split()[0] for l in text if l.strip() and not l.strip().endswith(">:") and " " in l.strip() and not l.strip().startswith(("Disassembly", ";"))]
        kinds = {}
        for i in ins:
            k = i.split("_")[0]
            kinds[k] = kinds.get(k, 0) + 1
        print(co, "static instructions:", len(ins), dict(sorted(kinds.items(), key=lambda x: -x[1])))
        note = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        for key in (".vgpr_count", ".sgpr_count", ".group_segment_fixed_size", ".private_segment_fixed_size",
                    ".vgpr_spill_count", ".sgpr_spill_count"):
            for l in note.splitlines():
                if key + ":" in l:
                    print("  ", l.strip())


if __name__ == "__main__":
    main()
