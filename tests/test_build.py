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


def _gen_lib(tmp_path, cxx, name):
    so = tmp_path / name
    subprocess.run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-o", str(so),
                    os.path.join(ROOT, "pollnet_amd", "csrc", "framegen.cpp"), "-L" + os.path.join(ROOT, "pollnet_amd"),
                    "-lpollnet_amd", "-lpthread", "-Wl,-rpath," + os.path.join(ROOT, "pollnet_amd")],
                   check=True, capture_output=True, timeout=300)
    return str(so)


def _gen(so, cfg, n, first=0):
    import ctypes

    import numpy as np

    import pollnet_amd as pa

    lib = ctypes.CDLL(so)
    p = pa.rx.GenParams.for_config(cfg)._c()
    out = np.empty((n, 2048), np.uint8)
    rc = lib.pn_gen_frames(ctypes.byref(p), ctypes.c_uint64(first), ctypes.c_uint32(n),
                           ctypes.c_void_p(out.ctypes.data), ctypes.c_uint32(2048), ctypes.c_uint32(2), ctypes.c_int(4))
    assert rc == 0
    return out


def test_generator_is_compiler_independent(tmp_path):
    """The seeded generator (framegen.cpp) draws one RNG value per statement, so its frames do not
    depend on the compiler's argument evaluation order (g++ evaluates right to left, clang left to
    right): built with both, it reproduces the committed slices' slot digests for C2..C5, and the two
    builds agree on 256 Ki frames of C3 and C5 (random miss flows and damaged payload bytes included)."""
    import hashlib
    import sys

    import numpy as np

    sys.path.insert(0, ROOT)
    golden = np.load(os.path.join(ROOT, "tests", "golden", "config_slices.npz"))
    libs = {cxx: _gen_lib(tmp_path, path, f"libgen_{cxx}.so")
            for cxx, path in (("gcc", "g++"), ("clang", "/opt/rocm/lib/llvm/bin/clang++"))}
    for cfg in (2, 3, 4, 5):
        for cxx, so in libs.items():
            s = _gen(so, cfg, 4096)
            assert hashlib.sha256(s.tobytes()).hexdigest() == str(golden[f"c{cfg}_slots_sha256"]), (cxx, cfg)
    for cfg in (3, 5):
        a, b = (_gen(so, cfg, 1 << 18, first=1 << 20) for so in libs.values())
        assert np.array_equal(a, b), cfg


def test_debug_dump_compiles(tmp_path):
    """Conn::dump / shortDump exist only under EFVITCP_DEBUG (as TcpConn.h:107-128): the debug build of a server
    and a client that call them compiles (hipcc, host and gfx950 device passes, syntax only)."""
    tu = tmp_path / "dump.cpp"
    tu.write_text("""#define EFVITCP_DEBUG
#include "pollnet_amd/tcp_server.hpp"
#include "pollnet_amd/tcp_client.hpp"
struct C {
  static const uint32_t RecvBufSize = 4096;
  static const uint32_t MaxConns = 4;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 0;
  static const uint32_t ConnSendBufCnt = 8;
  struct UserData {};
};
void f(const pollnet_amd::GpuTcpServer<C>::Conn& c) { c.dump("x"); c.shortDump("y"); }
void g(const pollnet_amd::GpuTcpClient<C>::Conn& c) { c.dump("x"); c.shortDump(); }
""")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                        "-fsyntax-only", "-x", "hip", str(tu)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
