"""Hashes of the shipped kernels' instruction streams in the built product library (no GPU needed).

The gfx950 code objects of xsknet_amd/libxsknet_amd.so (its .hip_fatbin offload bundles) are disassembled with
llvm-objdump; each kernel's instruction text (the encodings and address comments dropped: branch offsets are relative)
is hashed.  tests/golden/kernel_isa.json pins the transform kernels -- echo_round_kernel (launched, reference and wire
mode, large and small batches) and lowlat_kernel (the resident doorbell kernel, both modes) -- so that a source change
meant to leave them alone (pruning dead switches from xsk_echo_device.h) is checked to be
byte-identical in the built code, and a change meant to alter them updates the manifest deliberately:

    python tools/isa_manifest.py            # print every kernel's hash
    python tools/isa_manifest.py --check    # compare the pinned kernels with tests/golden/kernel_isa.json
    python tools/isa_manifest.py --write    # re-pin them (after an intended kernel change)
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.test_lowlat_isa import LIB, LLVM, gfx950_code_objects  # noqa: E402

MANIFEST = os.path.join(ROOT, "tests", "golden", "kernel_isa.json")
PINNED = re.compile(r"echo_round_kernel|lowlat_kernel")


def kernel_hashes(lib=LIB):
    """{demangled kernel name: (sha256-16 of its instruction text, instruction count)} of every kernel in `lib`."""
    funcs = {}
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(gfx950_code_objects(lib)):
            p = os.path.join(td, f"co{k}.o")
            open(p, "wb").write(co)
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", p], capture_output=True, text=True,
                                 check=True).stdout
            cur = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]{16} <(\S+)>:", line)
                if m:
                    cur = m.group(1)
                    funcs[cur] = []
                elif cur and line.startswith("\t"):
                    funcs[cur].append(line.split("//")[0].strip())
    names = subprocess.run(["c++filt"], input="\n".join(funcs), capture_output=True, text=True,
                           check=True).stdout.splitlines()
    return {dm: (hashlib.sha256("\n".join(ins).encode()).hexdigest()[:16], len(ins))
            for dm, ins in zip(names, funcs.values())}


def pinned(hashes):
    return {k: {"sha": v[0], "instructions": v[1]} for k, v in sorted(hashes.items()) if PINNED.search(k)}


def main(argv):
    h = kernel_hashes()
    if "--write" in argv:
        json.dump(pinned(h), open(MANIFEST, "w"), indent=1)
        print(f"wrote {MANIFEST}")
    elif "--check" in argv:
        want = json.load(open(MANIFEST))
        got = pinned(h)
        bad = {k for k in set(want) | set(got) if want.get(k) != got.get(k)}
        for k in sorted(bad):
            print("DIFFERS:", k, want.get(k), got.get(k))
        return 1 if bad else 0
    else:
        for k, (sha, n) in sorted(h.items()):
            print(sha, n, k)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
