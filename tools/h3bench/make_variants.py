"""Build h3bench once per ablation of csrc/h3_device.h (profiling tool; the product header is not modified).

Each variant replaces one component of latLngToCellDeg with a trivial stand-in so that
T(base) - T(variant) estimates that component's share of the kernel time on the GPU.
usage: python tools/h3bench/make_variants.py   (writes tools/h3bench/build/h3bench_<variant>)
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "..", "real-time-mobility-heatmap_amd", "csrc")
BUILD = os.path.join(HERE, "build")

X87_PLAIN = [("#define XMUL(a, K) xmul((a), HM_LD_##K##_M, HM_LD_##K##_E, HM_LD_##K##_HI, HM_LD_##K##_LO)",
              "#define XMUL(a, K) ((a) * HM_LD_##K##_HI)"),
             ("#define XADD(a, neg, K) xadd((a), (neg), HM_LD_##K##_M, HM_LD_##K##_E, HM_LD_##K##_HI, HM_LD_##K##_LO)",
              "#define XADD(a, neg, K) ((neg) ? (a) - HM_LD_##K##_HI : (a) + HM_LD_##K##_HI)")]
TRIG_CHEAP = [("    sincos(glat, &slat, &clat);", "    slat = glat; clat = 1.0 - glat * glat;"),
              ("    sincos(glng, &slng, &clng);", "    slng = glng; clng = 1.0 - glng * glng;"),
              ("    double r = acos(1 - sqd / 2);", "    double r = sqd;"),
              ("        sincos(dlng, &sd, &cd);", "        sd = dlng; cd = 1.0 - dlng;"),
              ("        double az = atan2(num, t1 - t2);", "        double az = num - t1 + t2;"),
              ("        r = tan(r);", "        r = r * 1.5;"),
              ("        sincos(theta, &st, &ct);", "        st = theta; ct = 1.0 - theta;")]
VARIANTS = {
    "base": [],
    "x87_plain": X87_PLAIN,
    "trig_cheap": TRIG_CHEAP,
    "face1": [("        for (int f = 0; f < 20; ++f) {\n            const float d", "        for (int f = 0; f < 1; ++f) {\n            const float d")],
    "no_rot": [("    if (T.baseCellData[baseCell][4]) {", "    if (false) {"),
               ("        for (int i = 0; i < k; i++) h = rotate60(h, cw);", "")],
    "no_digits": [("    for (int r = res - 1; r >= 0; r--) {", "    for (int r = -1; r >= 0; r--) {")],
    "x87_plain+trig_cheap": X87_PLAIN + TRIG_CHEAP,
}
# occupancy variants of the unmodified header: waves per SIMD (amdgpu_waves_per_eu) of the cells kernel
WAVES = {"base": 3, "base_w4": 4, "base_w5": 5, "base_w6": 6, "base_w8": 8}


def main():
    os.makedirs(BUILD, exist_ok=True)
    src = open(os.path.join(CSRC, "h3_device.h")).read()
    for name in list(WAVES) + [v for v in VARIANTS if v != "base"]:
        patches = VARIANTS.get(name, [])
        s = src
        for a, b in patches:
            if a not in s:
                sys.exit(f"{name}: pattern not found: {a}")
            s = s.replace(a, b)
        d = os.path.join(BUILD, name.replace("+", "_"))
        os.makedirs(d, exist_ok=True)
        open(os.path.join(d, "h3_device.h"), "w").write(s)
        for f in ("kernels.h", "h3_tables.inc", "h3_tables_host.h"):
            dst = os.path.join(d, f)
            if os.path.exists(dst):
                os.remove(dst)
            os.symlink(os.path.abspath(os.path.join(CSRC, f)), dst)
        out = os.path.join(BUILD, "h3bench_" + name.replace("+", "_"))
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               f'-DVARIANT="{name}"', f"-DH3B_WAVES={WAVES.get(name, 3)}", "-I", d, "-o", out, os.path.join(HERE, "h3bench.hip")]
        subprocess.run(cmd, check=True)
        print("built", out)


if __name__ == "__main__":
    main()
