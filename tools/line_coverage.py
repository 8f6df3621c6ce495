"""Statement coverage of the CPU test tier without coverage.py (not installed in this image).

Runs pytest in-process under a ``sys.settrace`` line tracer restricted to the package, main.py
and neural_net_model.py, and counts a file's executable lines as the line numbers carried by its
code objects (``co_lines``), i.e. the statements coverage.py measures. Python subprocesses (the
multi-rank gloo tests' ranks, the REST service's worker ranks) are traced too: a
``usercustomize`` hook (tools/_covhook) on their PYTHONPATH records their lines and the hits are
merged. Files listed under ``omit`` in .coveragerc are skipped like coverage.py skips them.
Prints a per-file table and the total, which is what ``fail_under`` in .coveragerc is checked
against.

    python tools/line_coverage.py [pytest args...]      (default: tests -q -m "not gpu")

GPU tier (on an MI355X): ``PZ_COV_GPU=1 python tools/line_coverage.py tests -q`` runs BOTH tiers
and also measures the GPU-only modules .coveragerc omits from the CPU gate (engine/*,
ops/functional.py); the CPU gate (fail_under) is not applied to that run.
"""
from __future__ import annotations

import configparser
import fnmatch
import glob
import json
import os
import sys
import tempfile
import threading
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sources() -> list[str]:
    cfg = configparser.ConfigParser()
    cfg.read(os.path.join(ROOT, ".coveragerc"))
    omit = [p.strip() for p in cfg.get("run", "omit", fallback="").splitlines() if p.strip()]
    if os.environ.get("PZ_COV_GPU") == "1":  # GPU tier: the fused engine and the autograd ops count
        omit = [p for p in omit if not (p.endswith("engine/*") or p.endswith("ops/functional.py"))]
    files = [os.path.join(ROOT, "main.py"), os.path.join(ROOT, "neural_net_model.py")]
    for d, _, names in os.walk(os.path.join(ROOT, "penr_oz_neural_network_torch_amd")):
        files += [os.path.join(d, n) for n in names if n.endswith(".py")]
    rel = lambda f: os.path.relpath(f, ROOT)
    return sorted(f for f in files if not any(fnmatch.fnmatch(rel(f), p) for p in omit))


def _executable(path: str) -> set[int]:
    src = open(path, encoding="utf-8").read()
    lines: set[int] = set()

    def walk(co: types.CodeType) -> None:
        for _, _, line in co.co_lines():
            if line is not None:
                lines.add(line)
        for c in co.co_consts:
            if isinstance(c, types.CodeType):
                walk(c)
    walk(compile(src, path, "exec"))
    # coverage.py's default exclusion: a line marked `# pragma: no cover` — and, when it opens a
    # block (`if ...:`, `def ...:`, `except ...:`), every line of that block — is not a statement
    text = src.splitlines()
    i = 0
    while i < len(text):
        line = text[i]
        if "pragma: no cover" in line:
            lines.discard(i + 1)
            code = line.split("#", 1)[0].rstrip()
            if code.endswith(":"):
                indent = len(line) - len(line.lstrip())
                j = i + 1
                while j < len(text) and (not text[j].strip() or len(text[j]) - len(text[j].lstrip()) > indent):
                    lines.discard(j + 1)
                    j += 1
                i = j
                continue
        i += 1
    return lines


def main(argv: list[str]) -> int:
    import pytest

    files = set(_sources())
    hit: dict[str, set[int]] = {f: set() for f in files}

    def tracer(frame, event, arg):
        f = frame.f_code.co_filename
        if f not in files:
            return None
        if event == "line":
            hit[f].add(frame.f_lineno)
        return tracer

    def global_tracer(frame, event, arg):
        if frame.f_code.co_filename in files:
            hit[frame.f_code.co_filename].add(frame.f_lineno)
            return tracer
        return None

    sub_dir = tempfile.mkdtemp(prefix="pz_linecov_")
    hook = os.path.join(ROOT, "tools", "_covhook")
    os.environ["PZ_LINECOV_DIR"] = sub_dir
    os.environ["PZ_LINECOV_FILES"] = json.dumps(sorted(files))
    os.environ["PYTHONPATH"] = hook + (os.pathsep + os.environ["PYTHONPATH"] if os.environ.get("PYTHONPATH") else "")
    if os.environ.get("PZ_COV_GPU") == "1":
        # autograd runs CUDA backward passes on its own device threads, created in C++ where
        # threading.settrace never reaches: the GPU autograd Functions' backward() lines would read
        # as unexecuted. Single-threaded autograd runs them on the calling (traced) thread.
        import torch
        torch.autograd.set_multithreading_enabled(False)
    sys.settrace(global_tracer)
    threading.settrace(global_tracer)
    try:
        rc = pytest.main(argv or ["tests", "-q", "-m", "not gpu", "-p", "no:cacheprovider"])
    finally:
        sys.settrace(None)
        threading.settrace(None)
    n_sub = 0
    for path in glob.glob(os.path.join(sub_dir, "*.json")):
        with open(path) as fh:
            for f, lines in json.load(fh).items():
                if f in hit:
                    hit[f].update(lines)
        n_sub += 1
    print(f"(merged line hits of {n_sub} traced subprocesses)")
    total_exec = total_hit = 0
    rows = []
    for f in sorted(files):
        ex = _executable(f)
        h = hit[f] & ex
        total_exec += len(ex)
        total_hit += len(h)
        rows.append((os.path.relpath(f, ROOT), len(ex), len(h)))
    print(f"\n{'file':64} {'stmts':>6} {'hit':>6} {'cover':>6}")
    for name, n, h in rows:
        print(f"{name:64} {n:6d} {h:6d} {100.0 * h / max(n, 1):5.1f}%")
    pct = 100.0 * total_hit / max(total_exec, 1)
    print(f"{'TOTAL':64} {total_exec:6d} {total_hit:6d} {pct:5.1f}%")
    if os.environ.get("PZ_LINECOV_MISSING"):  # show_missing: uncovered statement lines per file
        for f in sorted(files):
            miss = sorted(_executable(f) - hit[f])
            if miss:
                print(os.path.relpath(f, ROOT), ",".join(map(str, miss)))
    cfg = configparser.ConfigParser()
    cfg.read(os.path.join(ROOT, ".coveragerc"))
    gate = cfg.getfloat("report", "fail_under", fallback=0.0) if os.environ.get("PZ_COV_GPU") != "1" else 0.0
    if rc == 0 and pct < gate:
        print(f"FAIL: coverage {pct:.1f}% is below fail_under = {gate}")
        return 2
    return int(rc)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
