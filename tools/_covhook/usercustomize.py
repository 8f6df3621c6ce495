"""Subprocess half of tools/line_coverage.py: imported at interpreter start-up (``usercustomize``,
after the system's sitecustomize) in every Python child of a coverage run (multi-rank gloo tests,
the REST service's worker ranks), it records the executed lines of the measured files and dumps
them to ``$PZ_LINECOV_DIR/<pid>.json`` at exit. Inert unless PZ_LINECOV_DIR is set."""
import os

if os.environ.get("PZ_LINECOV_DIR"):
    import atexit
    import json
    import sys
    import threading

    _files = set(json.loads(os.environ.get("PZ_LINECOV_FILES", "[]")))
    _hits: dict = {}

    def _local(frame, event, arg):
        if event == "line":
            _hits.setdefault(frame.f_code.co_filename, set()).add(frame.f_lineno)
        return _local

    def _global(frame, event, arg):
        f = frame.f_code.co_filename
        if f in _files:
            _hits.setdefault(f, set()).add(frame.f_lineno)
            return _local
        return None

    sys.settrace(_global)
    threading.settrace(_global)

    def _dump():
        try:
            path = os.path.join(os.environ["PZ_LINECOV_DIR"], "%d.json" % os.getpid())
            with open(path, "w") as fh:
                json.dump({k: sorted(v) for k, v in _hits.items()}, fh)
        except OSError:
            pass

    atexit.register(_dump)
