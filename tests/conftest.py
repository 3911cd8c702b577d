import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "final-stage-path-tracer-2-0_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def _built():
    return all(os.path.exists(p) for p in (os.path.join(PKG, "libfsgpu.so"), os.path.join(PKG, "libfshost.so"),
                                           os.path.join(ORACLE, "liboracle.so")))


@pytest.fixture(scope="session", autouse=True)
def built_libs():
    if not _built():
        import subprocess

        subprocess.run(["make", "-s", "-j", "16", "-C", PKG], check=True)
        subprocess.run(["make", "-s", "-C", ORACLE], check=True)
    return True


@pytest.fixture(scope="session")
def scene_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("scenes"))


def load_scene(name, scene_dir):
    """Writes scene `name`, loads it through the C++ Scene mirror with the
    reference's RNG order (fresh stream, then InitializeMaterials)."""
    import fsamd
    import scenes

    path = scenes.write(name, os.path.join(scene_dir, name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(path)
    fsamd.initialize_materials()
    return s


@pytest.fixture(scope="session")
def _session_renderer():
    import fsamd

    if fsamd.device_count() < 1:
        pytest.fail("gpu test on a machine without a HIP device")
    r = fsamd.Renderer(0)
    yield r
    r.close()


@pytest.fixture
def gpu_renderer(_session_renderer):
    """The session's fs_context, back on fs_options_default() after each test."""
    import fsamd

    yield _session_renderer
    _session_renderer.set_options(**fsamd.options_dict(fsamd.options()))
