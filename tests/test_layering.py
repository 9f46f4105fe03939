"""The product never reaches the oracle: no import, no load, no fallback."""
import ast
import os

from conftest import REPO

PKG = os.path.join(REPO, "quantizations_amd")


def _py_files():
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith(".py"):
                yield os.path.join(root, f)


def test_product_does_not_import_oracle():
    for path in _py_files():
        tree = ast.parse(open(path).read())
        for node in ast.walk(tree):
            if isinstance(node, ast.Import):
                assert not any(a.name.split(".")[0] == "oracle" for a in node.names), path
            if isinstance(node, ast.ImportFrom):
                assert (node.module or "").split(".")[0] != "oracle", path


def test_product_sources_do_not_reference_oracle_library():
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                assert "liboracle" not in open(os.path.join(root, f)).read(), f


def test_missing_library_fails_loudly(tmp_path):
    import subprocess
    import sys

    env = dict(os.environ, QZ_LIB_PATH=str(tmp_path / "nope.so"), PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-c", "import quantizations_amd"], env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "libquantizations.so not found" in r.stderr
