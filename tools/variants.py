"""Builds kernel variants (-D flags) and benchmarks each in its own process.
   python tools/variants.py build name1="-DA -DB" name2="..."   (here)
   python tools/variants.py run name1 name2 ...                  (GPU box)"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "_variants")   # git-ignored, not gpurun-ignored: travels to the box

def build(specs):
    for spec in specs:
        name, flags = spec.split("=", 1)
        out = os.path.join(VDIR, f"librt_{name}.so")
        subprocess.run(["make", "-j8", f"OUT={out}", f"BUILD={VDIR}/{name}", f"EXTRA={flags}"],
                       cwd=os.path.join(ROOT, "raytracercpp_amd", "csrc"), check=True, capture_output=True)
        print("built", out, flush=True)

def run(names, extra):
    for name in names:
        env = dict(os.environ, RT_LIB_PATH=os.path.join(VDIR, f"librt_{name}.so"))
        r = subprocess.run([sys.executable, "bench.py", "--no-cpu-baseline"] + extra, cwd=ROOT, env=env,
                           capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(name, "FAILED", r.stderr[-2000:], flush=True)
            continue
        d = json.loads(line[-1])
        print(f"{name:16s} {d['value']:9.2f} Mrays/s  kernel {d['kernel_ms']:8.3f} ms  frac {d.get('roofline', {}).get('frac')}", flush=True)

if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        args = sys.argv[2:]
        extra = []
        if "--" in args:
            i = args.index("--"); extra = args[i + 1:]; args = args[:i]
        run(args, extra)
