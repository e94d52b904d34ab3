"""native.py's choice of HIP runtime (one runtime per process):
torch's bundled libamdhip64 is preloaded only when its ROCm major version
matches the build's /opt/rocm (or torch is already imported).  Host logic
only: nothing is loaded here."""

from teku_amd import native


def test_rocm_major_parsing():
    assert native._rocm_major("2.10.0+rocm7.0") == 7
    assert native._rocm_major("2.4.1+rocm6.1") == 6
    assert native._rocm_major("7.2.0") == 7
    assert native._rocm_major("6.4.3-123") == 6


def test_same_major_is_bool_and_matches_this_image():
    v = native._same_rocm_major()
    assert isinstance(v, bool)
    # this image: torch 2.10.0+rocm7.0 beside /opt/rocm 7.2.0 -> same major
    import importlib.metadata

    tv = importlib.metadata.version("torch")
    if "+rocm7" in tv:
        assert v
