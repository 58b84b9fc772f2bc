"""Static check of the gfx950 store-data hazard in a built library's device code.

A VMEM store of more than 64 bits (global_/buffer_/flat_store_dwordx3, _dwordx4) reads its data VGPRs
after it issues; a VALU instruction that writes one of those VGPRs within 2 wait states of the store
(gfx940+; LLVM GCNHazardRecognizer::createsVALUHazard / checkVALUHazardsHelper) can change the bytes the
store writes.  The compiler pads the stores it emits itself, but not a store written as inline asm --
it cannot see that the asm is a store -- so an asm `global_store_dwordx4` followed at once by a VALU
write of its data registers stores whatever the VALU wrote, for the lanes the store had not yet read.

This was the round-5 "wrong rows, not understood" pair: the inline-asm
non-temporal stores of st16_pol / st_chunk (gf_device.hpp), and two semantically equal variants of a
kernel body whose schedules happened to put a VALU write of a store's data right behind it.

Usage: python tools/store_hazard_check.py [library.so ...]   (default: chubaofs_amd/libcfsec.so)
Exit status 1 if any store is followed by a VALU write of its data within 2 wait states.
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

LLVM = "/opt/rocm/lib/llvm/bin"
WAIT_STATES = 2  # gfx940+ (VALUWaitStates in checkVALUHazardsHelper)

_STORE = re.compile(r"^\s*(global|buffer|flat|scratch)_store_dwordx([34])\s+(.*)$")
_INSN = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?\s*(?://.*)?$")
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def vregs(text):
    """VGPR numbers named by one operand."""
    out = set()
    for m in _VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def split_ops(s):
    ops, depth, cur = [], 0, ""
    for ch in s:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


def store_data_regs(mnemonic_family, ops):
    # global_store_dwordx4 vaddr, vdata, saddr|off ; buffer_store_dwordx4 vdata, vaddr, srsrc, soffset
    if mnemonic_family in ("global", "flat", "scratch"):
        return vregs(ops[1]) if len(ops) > 1 else set()
    return vregs(ops[0]) if ops else set()


def parse(lines):
    """Instructions of one disassembly: (address, mnemonic, operands, function, text, branch target)."""
    fn = "?"
    insns = []
    for line in lines:
        if re.match(r"^[0-9a-f]+ <.*>:$", line):
            fn = line.split("<", 1)[1].rstrip(">:")
            continue
        am = re.search(r"//\s*([0-9A-F]{6,}):", line)
        m = _INSN.match(line.split("//")[0])
        if not m or not am:
            continue
        tm = re.search(r"<(\S+)\+0x([0-9a-f]+)>", line)
        insns.append((int(am.group(1), 16), m.group(1), m.group(2) or "", fn, line.split("//")[0].strip(),
                      (tm.group(1), int(tm.group(2), 16)) if tm else None))
    return insns


def scan(lines):
    """Yield (function, store, offending instruction) for every store followed by a VALU write of its
    data within WAIT_STATES wait states, on the fall-through path and on branch targets."""
    insns = parse(lines)
    index = {a: i for i, (a, *_rest) in enumerate(insns)}
    fstart = {}
    for a, _mn, _o, fn, _t, _b in insns:
        fstart.setdefault(fn, a)

    def walk(i, ws, data, seen):
        while i < len(insns) and ws < WAIT_STATES:
            if i in seen:
                return
            seen.add(i)
            _a, mn, ops_s, fn, text, tgt = insns[i]
            if mn == "s_nop":
                ws += int(ops_s.split()[0], 0) + 1
                i += 1
                continue
            if mn in ("s_endpgm", "s_setpc_b64", "s_endpgm_saved"):
                return
            if mn.startswith("v_") and mn != "v_nop":
                ops = split_ops(ops_s)
                if ops and vregs(ops[0]) & data:
                    yield fn, text
            ws += 1
            if mn.startswith("s_cbranch") or mn == "s_branch":
                if tgt and tgt[0] in fstart and fstart[tgt[0]] + tgt[1] in index:
                    yield from walk(index[fstart[tgt[0]] + tgt[1]], ws, data, set(seen))
                if mn == "s_branch":
                    return
            i += 1

    for i, (_a, mn, ops_s, fn, text, _t) in enumerate(insns):
        sm = re.match(r"^(global|buffer|flat|scratch)_store_dwordx([34])$", mn)
        if not sm:
            continue
        data = store_data_regs(sm.group(1), split_ops(ops_s))
        for fn2, bad in walk(i + 1, 0, data, set()):
            yield fn, text, bad


def disassemble(so):
    tmp = tempfile.mkdtemp(prefix="hazchk")
    try:
        lib = os.path.join(tmp, os.path.basename(so))
        shutil.copy(so, lib)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        objs = [os.path.join(tmp, f) for f in sorted(os.listdir(tmp)) if "amdgcn" in f]

        def dis(path):
            r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", path], check=True,
                               capture_output=True, text=True)
            return r.stdout.splitlines()

        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            return list(ex.map(dis, objs))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def check(so):
    stores, bad = 0, []
    for lines in disassemble(so):  # one code object each (addresses restart)
        stores += sum(1 for l in lines if re.search(r"\b(global|buffer|flat)_store_dwordx[34]\b", l))
        bad.extend(scan(lines))
    return stores, bad


def main(argv):
    libs = argv or [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "chubaofs_amd",
                                 "libcfsec.so")]
    rc = 0
    for so in libs:
        stores, bad = check(so)
        print(f"{so}: {stores} stores of > 64 bits, {len(bad)} followed by a VALU write of their data "
              f"within {WAIT_STATES} wait states")
        for fn, st, v in bad[:40]:
            print(f"  {fn}\n    {st}\n    {v}")
        rc |= 1 if bad else 0
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
