"""The source-compatible C++ facade (include/PiXiuCtrl.h): client code written for
the reference's PiXiuCtrl compiles unchanged and runs on the GPU core."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(src, out):
    lib = os.path.join(ROOT, "pixiu_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), src, "-o", out,
                    "-L", lib, "-lpixiu_amd", f"-Wl,-rpath,{lib}"], check=True)


def test_facade(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path / "facade_test")
    _build(os.path.join(ROOT, "tests", "cpp", "facade_test.cpp"), exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "facade_test: ok" in r.stdout


def test_cli_transcript(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path / "pixiu_cli")
    _build(os.path.join(ROOT, "tools", "pixiu_cli.cpp"), exe)
    script = ("GET 123\nSET 123::321\nGET 123\nSET BOBO::https://www.zhihu.com/question/55439090\n"
              "SET BOBO1::https://www.zhihu.com/question/22454692\nGET BOBO\nGET BOBO1\n~\n")
    r = subprocess.run([exe], input=script, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "saved 27" in out  # README.md:85-87
    assert "123::321" in out and "BOBO1::https://www.zhihu.com/question/22454692" in out
