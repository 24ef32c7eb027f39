"""Ablation of the scene kernels (diagnostic builds, never shipped).

    python scripts/diag_variants.py build     # here: compiles the variants
    python scripts/diag_variants.py run       # GPU box: times each variant

Variants: SPRAY_DIAG_MODE=1 (domain mask only), 2 (mask + ordered domain
selection, no BVH), and the shipped kernel.  Prints the bench's per-kernel
milliseconds for each.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
DIAG = os.path.join(ROOT, "spray_amd", "lib", "diag")
VARIANTS = {"mask_only": ["SPRAY_DIAG_MODE=1"], "mask_select": ["SPRAY_DIAG_MODE=2"]}
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


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
