"""build() on a tree without the reference: the GPU box gets this tree minus the extracted
reference text (.gpurunignore: oracle/_ref/*.inc) and has no /root/reference, so `make` there
must keep the prebuilt example-handler tests instead of trying to recreate their input."""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_make_without_reference_or_extracted_text(tmp_path):
    dst = tmp_path / "tree"
    # copy2 keeps mtimes, as the snapshot that travels to the box does
    shutil.copytree(ROOT, dst, ignore=shutil.ignore_patterns(".git", "gpurun_out", "__pycache__", "*.inc"),
                    symlinks=True)
    assert not list((dst / "oracle" / "_ref").glob("*.inc"))
    r = subprocess.run(["make", "-C", str(dst), "REFDIR=/nonexistent", "-j4"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    for exe in ("tests/cpp/test_tcp_server", "tests/cpp/test_tcp_client_server", "bench/bench_tcp_server"):
        assert (dst / exe).exists(), exe  # prebuilt binaries kept
    # nothing left to do: a second make is a no-op
    r = subprocess.run(["make", "-C", str(dst), "REFDIR=/nonexistent", "-q", "pollnet_amd/libpollnet_amd.so",
                        "oracle/liboracle.so"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


def test_host_programs_build_for_gfx950_only():
    """Every hipcc line of the Makefile names the target arch (no default-arch device pass)."""
    with open(os.path.join(ROOT, "Makefile")) as f:
        text = f.read()
    assert "HOSTHIP = $(HIPCC) --offload-arch=$(ARCH)" in text
    for line in text.splitlines():
        if line.startswith("\t$(HIPCC)"):
            assert "$(HIPFLAGS)" in line, line
