"""Identity of the gfx950 kernels inside a built library: sha256 of each kernel's machine code.

The committed rocprofv3 --pmc traffic (profiles/pmc_traffic.json) is a measurement of particular kernel
code.  Each entry records, for every kernel its counters were summed over, the hash of that kernel's code
bytes in the library that ran; bench.py reports an entry's traffic only while the built library still holds
the same code (otherwise `traffic` is null and `traffic_stale` true), and tests/test_pmc_identity.py fails
when a production kernel changed without a PMC refresh.

The code object is found in the library's HIP fat binary (`.hip_fatbin`: a clang offload bundle, one entry
per target), its ELF symbol table gives each kernel's address and size, and the names are demangled with
c++filt to the form rocprofv3 prints in Kernel_Name.  Host-side only; reads the file, loads nothing."""
import functools
import hashlib
import os
import struct
import subprocess

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(blob: bytes, arch: str = "gfx950"):
    """The gfx950 code object of every offload bundle in the file (one per HIP translation unit)."""
    out = []
    i = blob.find(_BUNDLE_MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", blob, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if triple.startswith("hip") and arch in triple:
                out.append(blob[i + off:i + off + size])
        i = blob.find(_BUNDLE_MAGIC, i + 1)
    if not out:
        raise ValueError(f"no {arch} code object in the library")
    return out


def _elf_functions(elf: bytes):
    """{mangled name: code bytes} of the STT_FUNC symbols of a 64-bit little-endian ELF."""
    assert elf[:4] == b"\x7fELF" and elf[4] == 2 and elf[5] == 1, "not an ELF64 LE code object"
    e_shoff, = struct.unpack_from("<Q", elf, 0x28)
    e_shentsize, e_shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, e_shoff + k * e_shentsize) for k in range(e_shnum)]
    out = {}
    for name, typ, flags, addr, off, size, link, info, align, entsize in secs:
        if typ != 2:  # SHT_SYMTAB
            continue
        strtab = secs[link]
        for k in range(size // entsize):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf, off + k * entsize)
            if (st_info & 0xF) != 2 or st_size == 0 or st_shndx >= len(secs):  # STT_FUNC with code
                continue
            s0 = strtab[4] + st_name
            nm = elf[s0:elf.index(b"\0", s0)].decode()
            sec = secs[st_shndx]
            start = sec[4] + (st_value - sec[3])
            out[nm] = elf[start:start + st_size]
    return out


def _demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
    return r.stdout.splitlines()


@functools.lru_cache(maxsize=None)
def _kernel_hashes_cached(path: str, mtime_ns: int, size: int):
    with open(path, "rb") as f:
        blob = f.read()
    funcs = {}
    for co in _code_objects(blob):
        funcs.update(_elf_functions(co))
    names = sorted(funcs)
    return {d: hashlib.sha256(funcs[m]).hexdigest()[:16] for m, d in zip(names, _demangle(names))}


def kernel_hashes(path: str) -> dict:
    """{demangled kernel name (rocprofv3's Kernel_Name): sha256[:16] of its gfx950 machine code}."""
    st = os.stat(path)
    return dict(_kernel_hashes_cached(os.path.abspath(path), st.st_mtime_ns, st.st_size))


def product_library() -> str:
    return os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpollnet_amd.so")


def matching(names, path: str = None) -> dict:
    """{name: hash} for rocprofv3 kernel names; a name the library does not hold maps to None."""
    h = kernel_hashes(product_library())
    if path:
        h.update(kernel_hashes(path))
    return {n: h.get(n) for n in sorted(set(names))}


def check_entry(entry: dict, path: str = None):
    """(current, reason): whether a pmc_traffic.json entry's kernels are the built library's code."""
    ks = entry.get("kernels") if isinstance(entry, dict) else None
    if not ks:
        return False, "entry records no kernel code hashes"
    h = kernel_hashes(path or product_library())
    stale = [n for n, v in ks.items() if h.get(n) != v]
    if stale:
        return False, f"{len(stale)} of {len(ks)} kernels changed since the PMC run, e.g. {stale[0]}"
    return True, "kernel code identical to the PMC run's"
