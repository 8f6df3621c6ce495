"""One-GPU cost of the data-parallel step's collectives (VERDICT r3 missing #1 / next #4).

Runs bench.py (mlp4, the headline config) under each comm configuration on ONE MI355X and prints
ms/step, interleaved over rounds (same box):

  none          single process, no communication (the headline path: graph-free eager steps)
  torch         PZ_FORCE_COMM=1: a real 1-rank RCCL all-reduce per bucket via ProcessGroupNCCL
  native        PZ_FORCE_COMM=1 PZ_COMM=native: the extension's own RCCL communicator
  dpnone        PZ_FORCE_COMM=1 PZ_COMM=proxy with a zero-duration proxy: the DP schedule alone
  proxy_w<W>    PZ_COMM=proxy: the collective-footprint kernel (csrc/comm_proxy.hip) holds W
                channel workgroups for a modelled 8-rank ring all-reduce of every bucket at
                150 GB/s (the default schedule: full-grid tiled GEMMs)
  proxy_w<W>_sk the same with PZ_COMM_BUDGET=W: the backward GEMMs behind a bucket on the
                persistent stream-K engine with 256 - W CUs (parallel/dist.py comm_cus)
  zero_*        the same with the sharded optimizer (PZ_ZERO=1, engine/zero.py, default scope "mid":
                the weights complete mid-backward; zeroside_*: PZ_ZERO_SCOPE=side, + the paired
                partner; zeroall_*: PZ_ZERO_SCOPE=all, the first layer too): reduce-scatter +
                all-gather per weight (torch: real 1-rank RCCL calls, whole-weight slices; proxy:
                the modelled 8-rank world as its rank 0 — 1/8 of every weight updated, the proxy
                holding its workgroups for a ring reduce-scatter and a ring all-gather)

    python tools/comm_pressure.py [--rounds 2] [--steps 60] [--wgs 16,32]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(env_extra, steps, warmup):
    env = dict(os.environ, **env_extra)
    if env_extra.get("PZ_FORCE_COMM") == "1":  # a file rendezvous: no TCP port to race for
        import tempfile
        env["PZ_RENDEZVOUS_FILE"] = os.path.join(tempfile.mkdtemp(prefix="pz_rdv_"), "store")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(steps), "--warmup",
                          str(warmup)], env=env, capture_output=True, text=True, timeout=300)
    if out.returncode != 0:
        print(out.stderr[-2000:], file=sys.stderr)
        raise SystemExit(out.returncode)
    return json.loads(out.stdout.strip().splitlines()[-1])["ms_per_step"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--wgs", default="16,32")
    ap.add_argument("--gbps", default="150")
    ap.add_argument("--cases", default="", help="comma-separated subset of the case names")
    a = ap.parse_args()
    forced = {"PZ_FORCE_COMM": "1"}
    cases = {"none": {}, "torch": dict(forced, PZ_COMM="torch"), "native": dict(forced, PZ_COMM="native"),
             "dpnone": dict(forced, PZ_COMM="proxy", PZ_COMM_PROXY_GBPS="1e12")}
    for w in [int(x) for x in a.wgs.split(",")]:
        proxy = dict(forced, PZ_COMM="proxy", PZ_COMM_PROXY_WGS=str(w), PZ_COMM_PROXY_GBPS=a.gbps)
        cases[f"proxy_w{w}"] = proxy
        cases[f"proxy_w{w}_sk"] = dict(proxy, PZ_COMM_BUDGET=str(w))
        cases[f"zero_proxy_w{w}"] = dict(proxy, PZ_ZERO="1")
        cases[f"zeroall_proxy_w{w}"] = dict(proxy, PZ_ZERO="1", PZ_ZERO_SCOPE="all")
        cases[f"zeroside_proxy_w{w}"] = dict(proxy, PZ_ZERO="1", PZ_ZERO_SCOPE="side")
    cases["zero_torch"] = dict(forced, PZ_COMM="torch", PZ_ZERO="1")
    cases["zero_native"] = dict(forced, PZ_COMM="native", PZ_ZERO="1")
    cases["zero_dpnone"] = dict(cases["dpnone"], PZ_ZERO="1")
    cases["zeroall_dpnone"] = dict(cases["dpnone"], PZ_ZERO="1", PZ_ZERO_SCOPE="all")
    cases["zeroside_dpnone"] = dict(cases["dpnone"], PZ_ZERO="1", PZ_ZERO_SCOPE="side")
    for c in (x for x in a.cases.split(",") if x):
        if c not in cases:
            raise SystemExit(f"unknown case {c}: {sorted(cases)}")
    if a.cases:
        cases = {k: v for k, v in cases.items() if k in a.cases.split(",") or k == "none"}
    res = {name: [] for name in cases}
    for r in range(a.rounds):
        for name, env in cases.items():
            ms = run(env, a.steps, a.warmup)
            res[name].append(ms)
            print(f"round {r} {name:10s} {ms:.4f} ms/step", flush=True)
    base = min(res["none"])
    for name, v in res.items():
        print(f"{name:10s} best {min(v):.4f} ms  vs none {100 * (min(v) / base - 1):+.1f}%")


if __name__ == "__main__":
    main()
