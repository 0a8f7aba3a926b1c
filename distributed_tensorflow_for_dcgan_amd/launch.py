"""Single-node launcher with restart-based fault recovery.

    python -m distributed_tensorflow_for_dcgan_amd.launch --nproc 8 --max_restarts 3 -- \\
        image_train.py --data_dir=train --batch_size=128 ...

One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the env,
the same contract as ``torch.distributed.run``). When any rank exits non-zero, the launcher
stops the remaining ranks (each rank runs in its own process group; the launcher signals
exactly those groups), and -- up to ``--max_restarts`` times -- starts a fresh set of ranks on
a new rendezvous port. The trainer auto-resumes from the newest complete checkpoint (index
file written last), so a restart loses at most ``--save_model_secs`` of work. This replaces
the reference's "manual restart of the Supervisor" recovery, which could not actually resume
(no optimiser state in its checkpoints). A hung peer inside a collective is turned into an
error by the collective timeout (``--collective_timeout``), which then triggers the restart.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stop(procs: List[subprocess.Popen], grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t_end = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < t_end:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def _term_as_exit(signum, frame):
    raise SystemExit(128 + signum)


def launch(nproc: int, cmd: List[str], max_restarts: int = 0, master_addr: str = "127.0.0.1",
           master_port: int = 0, grace: float = 10.0, log=print) -> int:
    # the ranks run in their own sessions, so a SIGTERM to the launcher alone would orphan
    # them: turn it into an exception that stops them first
    try:
        signal.signal(signal.SIGTERM, _term_as_exit)
    except ValueError:  # not the main thread
        pass
    attempt = 0
    while True:
        port = master_port or _free_port()
        procs = []
        for r in range(nproc):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                       MASTER_ADDR=master_addr, MASTER_PORT=str(port), DCGAN_RESTART_COUNT=str(attempt))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
        log("[launch] attempt %d: %d ranks, rendezvous %s:%d" % (attempt, nproc, master_addr, port))
        failed = None
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    failed = bad[0]
                    break
                if all(c == 0 for c in codes):
                    log("[launch] all %d ranks finished" % nproc)
                    return 0
                time.sleep(0.1)
        except BaseException:  # SIGTERM (see _term_as_exit) / Ctrl-C: take the ranks down too
            _stop(procs, grace)
            raise
        log("[launch] rank %d exited with %d; stopping the other ranks" % failed)
        _stop(procs, grace)
        if attempt >= max_restarts:
            log("[launch] giving up after %d restart(s)" % attempt)
            return failed[1] if failed[1] > 0 else 1
        attempt += 1
        log("[launch] restart %d/%d (ranks resume from the newest checkpoint)" % (attempt, max_restarts))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--nproc", type=int, default=1, help="ranks (one per GPU)")
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("--master_addr", default="127.0.0.1")
    ap.add_argument("--master_port", type=int, default=0, help="0 = a free port per attempt")
    ap.add_argument("--grace", type=float, default=10.0, help="seconds between SIGTERM and SIGKILL")
    ap.add_argument("cmd", nargs=argparse.REMAINDER, help="-- script.py args...")
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing the command to launch")
    if cmd[0].endswith(".py"):
        cmd = [sys.executable] + cmd
    return launch(a.nproc, cmd, a.max_restarts, a.master_addr, a.master_port, a.grace,
                  log=lambda m: print(m, flush=True))


if __name__ == "__main__":
    sys.exit(main())
