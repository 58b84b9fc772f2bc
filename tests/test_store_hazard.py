"""The built library's device code has no store whose data registers a VALU instruction overwrites
within 2 wait states (the gfx940+ store-data hazard, tools/store_hazard_check.py).

Round 5 shipped two "wrong rows, not understood" results beside kernel bodies that passed every GPU
test: a compile-time output count in the fixed-K kernel gave (10, 4) / (12, 4)
StoreVerify a wrong second row, and a second instantiation of the lookup kernel's body wrong first rows
of each output quad.  The cause was the inline-asm stores of st16_pol / st_chunk: hipcc pads the
stores it emits itself but not an asm store, so those variants' schedules -- and six shipped (K, 1)
StoreVerify kernels -- put a VALU write of a store's data right behind it.  This check reads the
library's disassembly, so a schedule that brings the hazard back fails here on the CPU, whatever the
GPU tests happen to observe.  (The variants themselves: tools/r6_hazard_variants.py, measured on the
GPU in profiles/r06/hazard_variants.txt.)"""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "chubaofs_amd", "libcfsec.so")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists(LIB) or not shutil.which("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="needs the built library and llvm-objdump")
def test_no_store_data_hazard_in_library():
    import store_hazard_check as H
    stores, bad = H.check(LIB)
    assert stores > 1000, stores  # the disassembly was read
    assert not bad, "\n".join(f"{fn}: {st} / {v}" for fn, st, v in bad[:10])


def test_checker_flags_an_asm_store_followed_by_a_data_write():
    import store_hazard_check as H
    dis = """
0000000000001000 <k>:
	global_store_dwordx4 v[4:5], v[0:3], off nt                // 000000001000: DC7E8000 007F0004
	v_lshl_add_u64 v[0:1], s[0:1], 0, v[20:21]                 // 000000001008: D2080000 04510000
	global_store_dwordx4 v[4:5], v[8:11], off nt               // 000000001010: DC7E8000 007F0804
	s_nop 1                                                    // 000000001018: BF800001
	v_mov_b32_e32 v8, 0                                        // 00000000101C: 7E100280
	global_store_dwordx4 v[4:5], v[12:15], off nt              // 000000001020: DC7E8000 007F0C04
	v_mov_b32_e32 v0, 0                                        // 000000001028: 7E000280
	s_endpgm                                                   // 00000000102C: BF810000
""".splitlines()
    bad = list(H.scan(dis))
    assert len(bad) == 1 and "v_lshl_add_u64 v[0:1]" in bad[0][2]
