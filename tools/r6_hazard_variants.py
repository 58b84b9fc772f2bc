"""Builds the two round-5 "wrong rows, not understood" kernel variants, each with the round-5 inline-asm
stores (old) and with the round-6 hazard-free stores (new), into probes_bin/r6_hz/<variant>/libcfsec.so:

  A  the lookup-product kernel's chunk body called from a second, byte-path-free instantiation
     (gf_lut.hpp: lut_chunk<..., FULL = true> for whole chunks)
  B  the fixed-K kernel given the compile-time output count M instead of the launch's m (gf_device.hpp)
  C  neither (C_old: the current sources with the round-5 stores in every unit)

Every other unit is the current build (build/cfsec/*.o; run make first).  tools/store_hazard_check.py
then names the hazards of each library, and tools/r6_hazard_diag.py runs the failing shapes on a GPU.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result"]
UNITS = {"A": ["gf_lut_k6", "gf_lut_k12", "gf_lut_k15", "gf_lut_k16"],
         "C": [f[:-4] for f in sorted(os.listdir(os.path.join(ROOT, "chubaofs_amd", "csrc"))) if f.endswith(".hip")],
         "B": ["gf_k3", "gf_k4", "gf_k6", "gf_k7", "gf_k8", "gf_k10", "gf_k12", "gf_k15", "gf_k16", "gf_k18"]}


def patch_a(src):
    p = os.path.join(src, "gf_lut.hpp")
    s = open(p).read()
    a = ("template <int K, int M, int ML, MatVecMode MODE, int LA = CFSEC_LUT_LOOKAHEAD, int LW = 4>\n"
         "__device__ __forceinline__ void lut_chunk(")
    assert a in s
    s = s.replace(a, a.replace("int LW = 4>", "int LW = 4, bool FULL = false>"))
    b = "  const bool full = rem >= (uint32_t)NP;"
    assert b in s
    s = s.replace(b, "  const bool full = FULL || rem >= (uint32_t)NP;")
    c = ("    lut_chunk<K, M, ML, MODE, LA, LW>(reinterpret_cast<const char*>(T), tab01, tab2, in, out, "
         "(int)a.nstore, sbase, loff,\n                                      rem, diff);")
    assert c in s
    s = s.replace(c, "    if (rem == kLB)\n  " + c.replace("LA, LW>", "LA, LW, true>") + "\n    else\n  " +
                  c.replace("LA, LW>", "LA, LW, false>"))
    open(p, "w").write(s)


def patch_b(src):
    p = os.path.join(src, "gf_device.hpp")
    s = open(p).read()
    a = "lane_tile_k<K, M, MT, MODE, D, NTL, NTS, PAIR, LW, SP>((int)mrows, (int)a.nstore,"
    assert a in s
    s = s.replace(a, a.replace("(int)mrows", "M"))
    open(p, "w").write(s)


def old_stores(src):
    # the round-5 st16_pol / st_chunk (inline-asm stores, no wait states after them)
    old = subprocess.run(["git", "show", "7d54bbb:chubaofs_amd/csrc/gf_device.hpp"], cwd=ROOT, check=True,
                         capture_output=True, text=True).stdout
    cur = open(os.path.join(src, "gf_device.hpp")).read()
    i0, i1 = old.index("// 16-byte vector store with explicit"), old.index("// 16-byte load at base + off")
    j0, j1 = cur.index("// 16-byte vector store with explicit"), cur.index("// 16-byte load at base + off")
    cur = cur[:j0] + old[i0:i1] + cur[j1:]
    i0, i1 = old.index("template <int LW, bool NTS, int SP = CFSEC_STORE_POL>"), old.index("// Lane chunk of the fixed-K")
    j0, j1 = cur.index("template <int LW, bool NTS, int SP = CFSEC_STORE_POL>"), cur.index("// Lane chunk of the fixed-K")
    cur = cur[:j0] + old[i0:i1] + cur[j1:]
    open(os.path.join(src, "gf_device.hpp"), "w").write(cur)


def build(name):
    var, stores = name.split("_")
    work = f"/tmp/r6hz/{name}"
    shutil.rmtree(work, ignore_errors=True)
    src = os.path.join(work, "chubaofs_amd", "csrc")
    shutil.copytree(os.path.join(ROOT, "chubaofs_amd", "csrc"), src)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(work, "include"))
    if stores == "old":
        old_stores(src)
    if var != "C":  # C: the current sources (C_old: the round-5 stores in every unit, an A/B of the fix)
        (patch_a if var == "A" else patch_b)(src)
    out = os.path.join(ROOT, "probes_bin", "r6_hz", name)
    os.makedirs(out, exist_ok=True)
    def cc(u):
        o = os.path.join(work, u + ".o")
        subprocess.run([HIPCC, *FLAGS, "-c", os.path.join(src, u + ".hip"), "-o", o], check=True,
                       stderr=subprocess.DEVNULL)
        return o

    with ThreadPoolExecutor(max_workers=3) as ex:
        objs = list(ex.map(cc, UNITS[var]))
    objdir = os.path.join(ROOT, "build", "cfsec")
    objs += [os.path.join(objdir, f) for f in sorted(os.listdir(objdir)) if f[:-2] not in UNITS[var]]
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", os.path.join(out, "libcfsec.so"),
                    *objs], check=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{src}", os.path.join(ROOT, "tools", "gf_shapes.hip"),
                    f"-L{out}", "-lcfsec", "-Wl,-rpath,$ORIGIN", "-o", os.path.join(out, "gf_shapes")], check=True,
                   stderr=subprocess.DEVNULL)
    return out


if __name__ == "__main__":
    names = sys.argv[1:] or ["A_old", "A_new", "B_old", "B_new"]
    with ThreadPoolExecutor(max_workers=4) as ex:
        for o in ex.map(build, names):
            print(o)
