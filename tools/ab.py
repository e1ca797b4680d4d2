"""The one A/B driver: bench.py (or any command) under named variants, alternated, every run's
environment, library / source digests and result recorded.

    python tools/ab.py --out r06_x --reps 2 --steps 40 --workload cfg2 \\
        -v base: -v sk1:SCA_TNR_SK=1 -v prev:SCA_LIB_PATH=tools/lib_prev.so \\
        -v nofan:@ops._FAN_OUT=False

A variant is `name:` followed by comma-separated settings: `KEY=VALUE` sets an environment
variable for the run; `@module.attr=expr` overrides an attribute of scattennet_amd.ops /
keypoint_module / layers / attention before bench.py runs (tools/bench_var.py's mechanism).
--pre "pytest args" runs a GPU test subset once per variant first (a variant whose parity
fails is not timed).  Each run is under its own time limit and the first failure stops the
driver (GPU rules: no retries).  Output: gpurun_out/<out>/ab.json (every run: variant, rep,
env, digests, the bench line's value / ms_per_step / ms_per_step_median) and a summary table
on stdout (mean / min / max clips/s per variant, and the ratio to the first variant).
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_variant(spec):
    name, _, rest = spec.partition(":")
    env, attrs = {}, []
    for item in filter(None, (s.strip() for s in rest.split(","))):
        if item.startswith("@"):
            attrs.append(item[1:])
        else:
            k, _, v = item.partition("=")
            env[k] = v
    return {"name": name, "env": env, "attrs": attrs}


def digests(env):
    code = ("import os,sys; sys.path.insert(0, os.getcwd()); from scattennet_amd import _lib; "
            "print(_lib.source_digest()); print(_lib.library_digest())")
    try:
        out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                             timeout=120).stdout.split()
        return {"source_digest": out[0], "library_sources_digest": out[1]}
    except Exception as e:  # noqa: BLE001 — recorded, not fatal
        return {"digest_error": repr(e)}


def bench_cmd(v, args):
    bench = ["bench.py", "--steps", str(args.steps), "--warmup", str(args.warmup), "--no-cpu-baseline",
             "--workload", args.workload] + args.bench_args.split()
    if v["attrs"]:
        return [sys.executable, "tools/bench_var.py"] + v["attrs"] + ["--"] + bench[1:]
    return [sys.executable] + bench


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-v", "--variant", action="append", required=True, help="name:KEY=V,@ops.attr=expr")
    ap.add_argument("--out", default="ab")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--bench-args", default="", help="more bench.py arguments")
    ap.add_argument("--pre", default="", help="pytest arguments of a GPU test subset run once per variant")
    ap.add_argument("--timeout", type=int, default=300, help="seconds per run")
    args = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out", args.out)
    os.makedirs(out, exist_ok=True)
    variants = [parse_variant(s) for s in args.variant]
    runs = []
    for v in variants:
        v["full_env"] = dict(os.environ, **v["env"])
        v["digests"] = digests(v["full_env"])
        if args.pre:
            log = os.path.join(out, f"pre_{v['name']}.log")
            cmd = ["timeout", "-k", "10", str(args.timeout), sys.executable, "-u", "-m", "pytest", "-x", "-q",
                   "-p", "no:cacheprovider", "--timeout", "240", "--timeout-method", "thread"] + shlex.split(args.pre)
            with open(log, "w") as f:
                rc = subprocess.run(cmd, cwd=ROOT, env=v["full_env"], stdout=f, stderr=subprocess.STDOUT).returncode
            print(f"[{v['name']}] pre: rc={rc} {open(log).read().strip().splitlines()[-1:]}", flush=True)
            if rc != 0:
                sys.exit(rc)
    for rep in range(args.reps):
        for v in variants:
            log = os.path.join(out, f"{v['name']}_{rep}.log")
            t0 = time.time()
            with open(log, "w") as f:
                rc = subprocess.run(["timeout", "-k", "10", str(args.timeout)] + bench_cmd(v, args), cwd=ROOT,
                                    env=v["full_env"], stdout=f, stderr=subprocess.STDOUT).returncode
            line = next((json.loads(l) for l in open(log) if l.startswith('{"metric"')), None)
            rec = {"variant": v["name"], "rep": rep, "env": v["env"], "attrs": v["attrs"], **v["digests"],
                   "workload": args.workload, "steps": args.steps, "rc": rc, "wall_s": round(time.time() - t0, 1)}
            if line:
                rec.update({"value": line["value"], "ms_per_step": line["ms_per_step"],
                            "ms_per_step_median": line.get("ms_per_step_median")})
            runs.append(rec)
            json.dump(runs, open(os.path.join(out, "ab.json"), "w"), indent=1)
            print(f"[{v['name']} #{rep}] rc={rc} value={rec.get('value')} median_ms={rec.get('ms_per_step_median')}",
                  flush=True)
            if rc != 0 or line is None:
                print(open(log).read()[-2000:])
                sys.exit(rc or 1)
    base = None
    print(f"{'variant':<16}{'mean':>10}{'min':>10}{'max':>10}{'vs first':>10}")
    for v in variants:
        vals = [r["value"] for r in runs if r["variant"] == v["name"]]
        m = statistics.mean(vals)
        base = base or m
        print(f"{v['name']:<16}{m:>10.1f}{min(vals):>10.1f}{max(vals):>10.1f}{m / base:>10.4f}")


if __name__ == "__main__":
    main()
