import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# Parity gate (BASELINE.md "Parity gate"), fp32 engine vs float64 reference:
#   |ddB| <= 1e-3 for bins within 100 dB of the row peak, and
#   |d amplitude| <= 1e-5 * peak amplitude everywhere, amplitude = 10**(dB/20).
DB_TOL = 1e-3
DB_RANGE = 100.0
AMP_TOL = 1e-5


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def golden_cases():
    with open(os.path.join(GOLDEN, "cases.json")) as fh:
        return json.load(fh)


def golden_rows():
    return np.load(os.path.join(GOLDEN, "rows.npz"))


def window_of(w):
    return tuple(w) if isinstance(w, list) else w


def case_input(c):
    from pypanadapter_amd import synth
    if c.get("stored_input"):
        x = np.load(os.path.join(GOLDEN, "inputs.npz"))[c["name"]]
    else:
        x = synth.make_iq(c["n_samples"], c["fs"], c["seed"], n_fft=c["n_fft"], zoom=c["zoom"],
                          n_win=c["n_win"], f_lo=c["f_lo"], tones=c["tones"], noise=c["noise"])
    assert synth.digest(x) == c["input_sha256"], "synthetic generator drifted from the fixture"
    return x


def row_errors(row, ref):
    """(max |ddB| within DB_RANGE of the peak, max |d amp| / peak amp)."""
    row = np.asarray(row, np.float64)
    ref = np.asarray(ref, np.float64)
    fin = np.isfinite(ref)
    pk = ref[fin].max()
    m = fin & (ref > pk - DB_RANGE)
    ddb = float(np.abs(row - ref)[m].max())
    damp = float(np.abs(10 ** (row / 20.0) - 10 ** (ref / 20.0)).max() / 10 ** (pk / 20.0))
    return ddb, damp


# Tolerance ledger: the largest relative error each decimated-IQ check measured, by key, so the
# bounds can be set from measurements.  Written at the end of the session
# to $ZFFT_TOL_LEDGER when that is set (tools/gpu_session.sh "ledger").
_LEDGER = {}


def check_rel(got, ref, bound, key, what=""):
    """max |got - ref| / max |ref| < bound, recorded under `key`."""
    err = np.abs(np.asarray(got) - ref) / np.abs(ref).max()
    e = float(err.max())
    _LEDGER[key] = max(_LEDGER.get(key, 0.0), e)
    assert e < bound, (key, what, e, int(err.argmax()), len(err))
    return e


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("ZFFT_TOL_LEDGER")
    if path and _LEDGER:
        with open(path, "w") as fh:
            json.dump({k: _LEDGER[k] for k in sorted(_LEDGER)}, fh, indent=1)


def assert_row_close(row, ref, what="", db_tol=DB_TOL, amp_tol=AMP_TOL):
    ddb, damp = row_errors(row, ref)
    assert ddb <= db_tol and damp <= amp_tol, f"{what}: max|ddB|={ddb:.3e} max|damp|={damp:.3e}"


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import coracle
    coracle.build()
    return coracle


@pytest.fixture(scope="session")
def zfft_lib():
    from pypanadapter_amd import _lib, build
    build.build()
    return _lib.load()
