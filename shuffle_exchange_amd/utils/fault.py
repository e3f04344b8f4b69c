"""Fault injection for failure-handling tests (the reference has none).

``SXE_FAULT`` holds ``;``-separated rules ``<action>@<rank>:<step>``:
  * ``kill@1:3``  -- rank 1 exits with status 17 when the engine reaches global step 3
    (exercises the launcher's fail-fast teardown, launcher/launch.py);
  * ``hang@0:2``  -- rank 0 sleeps forever at step 2 (exercises collective timeouts /
    ``monitored_barrier``);
  * ``raise@2:5`` -- rank 2 raises ``InjectedFault`` at step 5 (exception paths, checkpoint
    recovery tests).
``rank`` may be ``*``. Collectives can additionally be turned into no-ops per kind through the
``SXE_COMM_<KIND>_OFF`` switches of comm/comm.py (the reference's ``DS_COMM_*_OFF``).
"""
import os
import sys
import time


class InjectedFault(RuntimeError):
    pass


def _rules():
    spec = os.environ.get("SXE_FAULT", "").strip()
    out = []
    for part in filter(None, (p.strip() for p in spec.split(";"))):
        action, _, where = part.partition("@")
        rank, _, step = where.partition(":")
        out.append((action.strip().lower(), rank.strip(), int(step)))
    return out


def maybe_inject(rank, step):
    for action, r, s in _rules():
        if s != step or (r != "*" and int(r) != rank):
            continue
        sys.stderr.write(f"[sxe fault] {action} on rank {rank} at step {step}\n")
        sys.stderr.flush()
        if action == "kill":
            os._exit(17)
        if action == "hang":
            while True:
                time.sleep(3600)
        if action == "raise":
            raise InjectedFault(f"injected fault on rank {rank} at step {step}")
