"""One host RX ring shared by the ranks of a node, sharded by index (the multi-GPU end-to-end leg).

The reference's ring is `RecvBufCnt` slots of `RecvBufSize` bytes in host memory that the NIC fills and
`Core::pollNet` walks (/root/reference/efvitcp/Core.h:140-145, 285-289).  Here the ring is one shared-memory
segment of `world * n_per_rank` slots plus one 16-B record per slot; rank r owns slots [r*n, (r+1)*n) and their
records.  Each rank
  - first-touches its own shard from CPUs of its GPU's NUMA node (the pages then live on that node, so the
    GPU reads them over its own PCIe root without crossing the socket link), and
  - registers only its shard and its records with HIP (hipHostRegister, mapped), so its GPU classifies the
    frames in place (zero copy: only the lines the kernel needs cross PCIe) and writes the records straight
    into the shared segment, where any process on the node reads them.
No collective and no exchange: the index shards are independent.  CPU-only parts (layout, NUMA
lookup, the shared mapping) run without a GPU; register() needs HIP."""
from __future__ import annotations

import contextlib
import ctypes
import os

import numpy as np

RECORD_BYTES = 16


def _cpulist(text: str):
    out = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def device_numa(pci_domain: int, pci_bus: int, pci_device: int):
    """(NUMA node, the node's CPUs this process may run on) of a PCI device, from sysfs; (-1, []) if unknown."""
    bdf = f"{pci_domain:04x}:{pci_bus:02x}:{pci_device:02x}.0"
    try:
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        return -1, []
    if node < 0:
        return node, []
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _cpulist(f.read())
    except OSError:
        return node, []
    allowed = os.sched_getaffinity(0)
    return node, [c for c in cpus if c in allowed]


@contextlib.contextmanager
def cpu_affinity(cpus):
    """Run the body (and the threads it starts) on `cpus`; unchanged when the list is empty."""
    if not cpus:
        yield
        return
    old = os.sched_getaffinity(0)
    os.sched_setaffinity(0, cpus)
    try:
        yield
    finally:
        os.sched_setaffinity(0, old)


def room_for(nbytes: int, shm_dir: str = "/dev/shm"):
    """None if a shared segment of nbytes fits both the shared-memory filesystem's free space and half the host's
    available memory, else the reason.  A tmpfs that fills up under a mapping kills the writer with SIGBUS, which
    no handler turns into an error, so the size is checked before anything is created."""
    try:
        st = os.statvfs(shm_dir)
        free = st.f_bavail * st.f_frsize
    except OSError as ex:
        return f"{shm_dir}: {ex}"
    if nbytes > free:
        return f"{shm_dir} has {free / 2**30:.1f} GiB free, the ring needs {nbytes / 2**30:.1f} GiB"
    try:
        with open("/proc/meminfo") as f:
            avail = next(int(ln.split()[1]) * 1024 for ln in f if ln.startswith("MemAvailable:"))
        if nbytes > avail // 2:
            return f"the ring ({nbytes / 2**30:.1f} GiB) exceeds half the host's available memory ({avail / 2**30:.1f} GiB)"
    except (OSError, StopIteration, ValueError):
        pass
    return None


class SharedHostRing:
    """world * n_per_rank slots of `stride` bytes, then world * n_per_rank 16-B records, in one POSIX
    shared-memory segment.  Collective over `dist` (torch.distributed or None for one process): rank 0
    checks the room (room_for), creates the segment and broadcasts its name; every rank maps all of it.  When
    there is no room every rank raises the same RuntimeError (nobody is left waiting)."""

    def __init__(self, dist, rank: int, world: int, n_per_rank: int, stride: int):
        import secrets
        from multiprocessing import shared_memory

        self.rank, self.world, self.n, self.stride = rank, world, n_per_rank, stride
        self.slot_bytes = world * n_per_rank * stride
        size = self.slot_bytes + world * n_per_rank * RECORD_BYTES
        name = [None, None]
        if rank == 0:
            name[1] = room_for(size)
            if name[1] is None:
                try:
                    name[0] = f"pn_ring_{secrets.token_hex(6)}"
                    self.shm = shared_memory.SharedMemory(name=name[0], create=True, size=size)
                except OSError as ex:
                    name = [None, f"creating the shared ring: {ex!r}"]
        if dist is not None and world > 1:
            dist.broadcast_object_list(name, src=0)
        if name[0] is None:
            raise RuntimeError(f"no shared host ring: {name[1]}")
        if rank != 0:
            self.shm = shared_memory.SharedMemory(name=name[0])
            from multiprocessing import resource_tracker

            resource_tracker.unregister(self.shm._name, "shared_memory")  # only the creator unlinks it
        self._registered = []
        self._hip = None

    # ---- layout
    def slots(self) -> np.ndarray:
        """The whole ring, (world * n, stride) bytes."""
        return np.ndarray((self.world * self.n, self.stride), dtype=np.uint8, buffer=self.shm.buf)

    def shard(self, rank: int = None) -> np.ndarray:
        r = self.rank if rank is None else rank
        return self.slots()[r * self.n:(r + 1) * self.n]

    def records(self, rank: int = None) -> np.ndarray:
        """Rank's records as bytes, n * 16 (pn_result each)."""
        r = self.rank if rank is None else rank
        all_rec = np.ndarray((self.world * self.n * RECORD_BYTES,), dtype=np.uint8, buffer=self.shm.buf,
                             offset=self.slot_bytes)
        return all_rec[r * self.n * RECORD_BYTES:(r + 1) * self.n * RECORD_BYTES]

    def addresses(self):
        """(shard address, records address) of this rank: host pointers a registered range is used through."""
        return self.shard().ctypes.data, self.records().ctypes.data

    # ---- HIP
    def register(self):
        """hipHostRegister (mapped) this rank's shard and records: the GPU then reads / writes them in place."""
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
        self._hip = hip
        for ptr, nbytes in ((self.shard().ctypes.data, self.n * self.stride),
                            (self.records().ctypes.data, self.n * RECORD_BYTES)):
            rc = hip.hipHostRegister(ptr, nbytes, 0x2)  # hipHostRegisterMapped
            if rc != 0:
                raise RuntimeError(f"hipHostRegister({nbytes} B of the shared ring) failed: hipError {rc}")
            self._registered.append(ptr)

    def close(self, dist=None):
        if self._hip is not None:
            for ptr in self._registered:
                self._hip.hipHostUnregister(ptr)
            self._registered = []
        if dist is not None and self.world > 1:
            dist.barrier()  # nobody uses the segment any more
        try:
            self.shm.close()
        except BufferError:  # a caller still holds a view: the mapping goes with the process
            pass
        if self.rank == 0:
            self.shm.unlink()
