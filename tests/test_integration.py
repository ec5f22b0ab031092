"""The drop-in boundary as the reference sees it (build container; needs /root/reference).

tests/integration_probe.py runs in a child process (it installs the gymnasium stub): the reference's
own registration.py + make_vec, with ap_gym_amd.integration.register_with_ap_gym() applied, must
return the backend env itself (a subclass of the reference's BaseActivePerceptionVectorEnv) with the
build's loss_fn and prediction spaces, and the registrations must satisfy gymnasium's rule against a
vector entry point with additional_wrappers (registration.py:124-125).
"""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reference_available():  # the probe and tests/golden/refload.py exist only in the build container
    ref = os.environ.get("APG_REFERENCE_ROOT", "/root/reference")
    return (os.path.isfile(os.path.join(ref, "ap_gym", "envs", "registration.py"))
            and os.path.isfile(os.path.join(ROOT, "tests", "integration_probe.py")))


@pytest.mark.skipif(not _reference_available(), reason="needs the reference tree (build container only)")
def test_reference_make_vec_returns_backend_env(oracle_mod):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "integration_probe.py")], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "integration probe OK" in r.stdout


def test_env_classes_are_vector_envs():
    """Without gymnasium the envs derive from the local VectorEnv stand-in; with it (the probe above)
    from gymnasium.vector.VectorEnv."""
    import ap_gym_amd as ap
    from ap_gym_amd.vector_env import VectorEnv

    for cls in (ap.LIDARLocalization2DVectorEnv, ap.ImageClassificationVectorEnv, ap.ImageLocalizationVectorEnv,
                ap.LightDarkVectorEnv, ap.CircleSquareHideAndSeekVectorWrapper):
        assert issubclass(cls, VectorEnv), cls
