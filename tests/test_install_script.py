"""install.sh (the reference's installer, /root/reference/install.sh:1-11): valid bash that builds the gfx950
library in-tree and installs the `xot` console script without network access."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_install_script_parses_and_builds_offline():
  path = os.path.join(ROOT, "install.sh")
  assert os.access(path, os.X_OK)
  subprocess.run(["bash", "-n", path], check=True)
  text = open(path).read()
  assert "build_ext --inplace" in text and "gfx950" in text
  assert "--no-index" in text  # never reaches for a package index
