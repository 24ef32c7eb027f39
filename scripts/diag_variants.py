"""Ablation of the scene kernels (diagnostic builds, never shipped).

    python scripts/diag_variants.py build     # here: compiles the variants
    python scripts/diag_variants.py run       # GPU box: times each variant
    python scripts/diag_variants.py check     # GPU box: AO parity tests per variant

Variants: SPRAY_DIAG_MODE=1 (domain mask only), 2 (mask + ordered domain
selection, no BVH), the any-hit variants of spray_amd/csrc/rt_kernels_diag.inc
(SPRAY_AH_SPREAD=1, SPRAY_AO_REFILL=32 -- re-packing schemes measured slower
than the shipped walk), and the shipped kernel.  "run" prints the bench's
per-kernel milliseconds for each; "check" runs tests/test_gpu_ao.py against
each any-hit variant (they must stay bit-exact).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DIAG = os.path.join(ROOT, "spray_amd", "lib", "diag")
VARIANTS = {"mask_only": ["SPRAY_DIAG_MODE=1"], "mask_select": ["SPRAY_DIAG_MODE=2"],
            "ah_spread": ["SPRAY_AH_SPREAD=1"], "ao_refill": ["SPRAY_AO_REFILL=32"],
            "aogroup": ["SPRAY_AO_GROUP=1"]}
CHECKED = ("ah_spread", "ao_refill", "aogroup")  # bit-exact variants: parity tests apply
EXTRA = dict(a.split("=", 1) for a in sys.argv[2:] if "=" in a)  # name=DEF1,DEF2


def build():
    from spray_amd import build as b
    b.build()
    v = dict(VARIANTS)
    for k, d in EXTRA.items():
        v[k] = d.split(",")
    for name, defs in v.items():
        print(b.build(defines=defs, out=os.path.join(DIAG, "libspray_rt_%s.so" % name)))


def run():
    libs = [("shipped", None)] + sorted(
        (f[len("libspray_rt_"):-3], os.path.join(DIAG, f)) for f in os.listdir(DIAG))
    for name, lib in libs:
        env = dict(os.environ)
        if lib:
            env["SPRAY_RT_LIB"] = lib
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "10",
                            "--warmup", "2", "--cpu-baseline", "0", "--frame", "0", "--ooc", "0"], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(name, "FAILED", r.returncode, r.stderr[-800:])
            continue
        j = json.loads(line[-1])
        print("%-14s step %.4f ms  ao %.4f ms  %s" % (name, j["ms_per_step"], j.get("ao", {}).get("ms_per_step", 0), json.dumps(j["kernels_ms"])),
              flush=True)


def check():
    bad = 0
    for name in CHECKED:
        lib = os.path.join(DIAG, "libspray_rt_%s.so" % name)
        env = dict(os.environ, SPRAY_RT_LIB=lib)
        r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "--timeout",
                            "300", os.path.join(ROOT, "tests", "test_gpu_ao.py")], env=env,
                           capture_output=True, text=True, timeout=900)
        print(name, "rc", r.returncode, r.stdout.strip().splitlines()[-1] if r.stdout else "",
              flush=True)
        bad += r.returncode != 0
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    {"build": build, "run": run, "check": check}[sys.argv[1]]()
