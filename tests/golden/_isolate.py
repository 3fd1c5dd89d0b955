"""Run a reference-fixture generator (make_ref_*.py) in a throwaway child process: the reference's
Python is untrusted input, so the child gets a scrubbed environment (no inherited variables beyond
the locale / hash seed the generators need), a temporary HOME and working directory that are deleted
afterwards, and no user site-packages (-s).  The committed .npz written into tests/golden/ is the only
artifact the tests consume; nothing else of the child's run is kept.  Build container only."""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

CHILD_FLAG = "DSSM_REF_FIXTURE_CHILD"


def in_child() -> bool:
    return os.environ.get(CHILD_FLAG) == "1"


def rerun_isolated(script: str, argv) -> int:
    with tempfile.TemporaryDirectory(prefix="dssm_ref_fixture_") as tmp:
        env = {CHILD_FLAG: "1", "PATH": "/usr/bin:/bin", "HOME": tmp, "TMPDIR": tmp,
               "PYTHONUTF8": "1", "PYTHONHASHSEED": "0", "LANG": "C.UTF-8"}
        return subprocess.run([sys.executable, "-s", os.path.abspath(script)] + list(argv), env=env,
                              cwd=tmp).returncode
