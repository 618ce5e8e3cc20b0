"""Cold start of the drop-in executable: bin/transfer llnl_slab_test.prm
(the reference's unit of use, src/main.cc:60-136: one process per .prm) from process start to
exit, and its split into phases by tools/transfer_phases (build: make -C radiative-transfer_amd
tools): exec -> main, the .prm, HIP init, create, the first solve, the read-outs, the CSV
files, a second create / solve / read-out in the same process, and the teardown after main.
Median of REPS fresh processes per configuration, with the HIP runtime's code-object loading
deferred (the default) and eager (HIP_ENABLE_DEFERRED_LOADING=0), and once with the
runtime's first-use costs (a stream, the first pinned copies each way, a pageable copy) timed
on their own before the library's first call.  JSON lines on stdout.
usage: python -u tools/transfer_phases.py [reps]"""
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
TRANSFER = REPO / "radiative-transfer_amd" / "bin" / "transfer"
PHASES = REPO / "tools" / "transfer_phases"
PRM = REPO / "tests" / "golden" / "prm"
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def run(cmd, env, cwd):
    t0 = time.monotonic_ns()
    r = subprocess.run(cmd + ([str(t0)] if cmd[0] == str(PHASES) else []), env=env, cwd=cwd, capture_output=True,
                       text=True, timeout=120)
    t1 = time.monotonic_ns()
    if r.returncode:
        raise RuntimeError(f"{cmd}: {r.returncode} {r.stderr[-500:]}")
    return t0, t1, r.stdout


for name in ("llnl_slab_test.prm", "single_group.prm"):
    for deferred, probe in (("1", False), ("1", True), ("0", False)):
        env = dict(os.environ, RT_TABLE_DIR=str(PRM) + "/", RTSN_QUIET="1", HIP_ENABLE_DEFERRED_LOADING=deferred)
        if not probe:
            env["PHASES_NO_PROBE"] = "1"
        walls, phases = [], []
        with tempfile.TemporaryDirectory() as cwd:
            for _ in range(REPS):
                t0, t1, _ = run([str(TRANSFER), str(PRM / name)], env, cwd)
                walls.append(1e-6 * (t1 - t0))
                t0, t1, out = run([str(PHASES), str(PRM / name)], env, cwd)
                d = json.loads(out.strip().splitlines()[-1])
                d["teardown_ms"] = 1e-6 * (t1 - d.pop("t_end_ns"))
                d["process_ms"] = 1e-6 * (t1 - t0)
                phases.append(d)
        med = {k: statistics.median(p[k] for p in phases) for k in phases[0] if k.endswith("_ms")}
        print(json.dumps({"prm": name, "HIP_ENABLE_DEFERRED_LOADING": deferred, "runtime_probes": probe, "reps": REPS,
                          "transfer_wall_ms": {"median": statistics.median(walls), "min": min(walls),
                                               "all": [round(w, 2) for w in walls]},
                          "phases_median_ms": {k: round(v, 4) for k, v in med.items()}}), flush=True)
