"""pytest configuration: import paths, the `gpu` marker and shared fixtures.

`-m "not gpu"` tests run on any CPU host (oracle vs golden vectors, loader, C-ABI exports);
`-m gpu` tests need an MI355X and compare the HIP path with the oracle (tests/README in
DESIGN.md section 6).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "complexity-tokenizer_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) -- parity tests of the HIP path")


def pytest_collection_finish(session):
    """A GPU session that will run the full-size digest tests (tests/test_gpu_z_full_configs.py)
    starts building their 1M-doc corpora in background processes now, before any test touches the
    GPU, so that they are ready when those tests (collected last) run."""
    names = {getattr(it, "callspec", None) and it.callspec.params.get("cfg") for it in session.items
             if it.module.__name__.endswith("test_gpu_z_full_configs")}
    names.discard(None)
    if names:
        from datagen import cache
        groups = [[n for n in ("C5", "C5NFC") if n in names or (n == "C5" and "C5NFC" in names)], ["C2"] if "C2" in names else []]
        cache.start_background(cache.default_dir(), [g for g in groups if g])


@pytest.fixture(scope="session")
def fixture_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("tokjson"))


@pytest.fixture(scope="session")
def gpt2_path(fixture_dir):
    from datagen.build_tokenizers import fixture_path
    return fixture_path("gpt2_50k", fixture_dir)


@pytest.fixture(scope="session")
def llama3_path(fixture_dir):
    from datagen.build_tokenizers import fixture_path
    return fixture_path("llama3_128k", fixture_dir)


@pytest.fixture(scope="session")
def multi_path(fixture_dir):
    from datagen.build_tokenizers import fixture_path
    return fixture_path("multi_32k", fixture_dir)



@pytest.fixture(scope="session")
def llama3_tt_path(fixture_dir):
    from datagen.build_tokenizers import fixture_path
    return fixture_path("llama3_tt_128k", fixture_dir)
