"""The feed path's host topology (host_numa.cpp), host-only: a GPU's NUMA node and CPU set are read
from sysfs through its PCI bus id, as nhip_init does for every context (the context then places its
pinned staging on that node and binds its staging copy threads to those CPUs).  Fixture sysfs trees
model an 8-GPU two-socket node (four GPUs per socket), a platform that reports no node (-1), a
missing device and malformed files; the kernel cpulist syntax is parsed as the kernel writes it."""
import ctypes
import os

import pytest

import neptune_hip._lib as L


def _lib():
    try:
        return L.load()
    except OSError as e:  # pragma: no cover - the build check covers a missing library
        pytest.skip(f"libneptune_hip.so not loadable: {e}")


def _topo(lib, root, bus):
    node = ctypes.c_int(-7)
    n = ctypes.c_size_t(0)
    rc = lib.nhip_numa_from_sysfs(str(root).encode(), bus.encode(), ctypes.byref(node), None, 0, ctypes.byref(n))
    assert rc == 0
    cpus = (ctypes.c_int * max(1, n.value))()
    got = ctypes.c_size_t(0)
    assert lib.nhip_numa_from_sysfs(str(root).encode(), bus.encode(), ctypes.byref(node), cpus, n.value,
                                    ctypes.byref(got)) == 0
    return node.value, list(cpus[:got.value])


def _write(path, text):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


# an MI355X node as the driver's 8-GPU runs would see it: two sockets of 96 cores (SMT siblings
# listed after the cores), GPUs 0-3 behind socket 0 and 4-7 behind socket 1
BUS = ["0000:05:00.0", "0000:15:00.0", "0000:65:00.0", "0000:75:00.0",
       "0000:85:00.0", "0000:95:00.0", "0000:E5:00.0", "0000:F5:00.0"]
NODE_CPUS = {0: "0-95,192-287\n", 1: "96-191,288-383\n"}


@pytest.fixture()
def two_socket(tmp_path):
    for i, b in enumerate(BUS):
        _write(tmp_path / "bus/pci/devices" / b.lower() / "numa_node", f"{0 if i < 4 else 1}\n")
    for n, lst in NODE_CPUS.items():
        _write(tmp_path / f"devices/system/node/node{n}/cpulist", lst)
    return tmp_path


def test_eight_gpus_map_to_their_sockets(two_socket):
    lib = _lib()
    want = {0: list(range(0, 96)) + list(range(192, 288)), 1: list(range(96, 192)) + list(range(288, 384))}
    for i, b in enumerate(BUS):
        node, cpus = _topo(lib, two_socket, b)
        assert node == (0 if i < 4 else 1)
        assert cpus == want[node]
    # hipDeviceGetPCIBusId may report upper-case hex; sysfs names are lower-case
    assert _topo(lib, two_socket, BUS[6])[0] == 1 and _topo(lib, two_socket, BUS[6].lower())[0] == 1


def test_no_node_reported_or_no_device(tmp_path):
    lib = _lib()
    _write(tmp_path / "bus/pci/devices/0000:05:00.0/numa_node", "-1\n")
    assert _topo(lib, tmp_path, "0000:05:00.0") == (-1, [])
    assert _topo(lib, tmp_path, "0000:99:00.0") == (-1, [])  # no such device
    _write(tmp_path / "bus/pci/devices/0000:06:00.0/numa_node", "garbage\n")
    assert _topo(lib, tmp_path, "0000:06:00.0") == (-1, [])
    # a node without a cpulist (memory-only node): the node, no CPUs to bind
    _write(tmp_path / "bus/pci/devices/0000:07:00.0/numa_node", "3\n")
    assert _topo(lib, tmp_path, "0000:07:00.0") == (3, [])


def _parse(lib, text):
    n = ctypes.c_size_t(0)
    rc = lib.nhip_cpulist_parse(text.encode(), None, 0, ctypes.byref(n))
    if rc:
        return None
    buf = (ctypes.c_int * max(1, n.value))()
    assert lib.nhip_cpulist_parse(text.encode(), buf, n.value, ctypes.byref(n)) == 0
    return list(buf[:n.value])


def test_cpulist_syntax():
    lib = _lib()
    assert _parse(lib, "0") == [0]
    assert _parse(lib, "0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert _parse(lib, "0-11:4") == [0, 4, 8]
    assert _parse(lib, "8-9,0-1,1") == [0, 1, 8, 9]  # sorted, deduplicated
    assert _parse(lib, "") == []
    for bad in ("a", "3-1", "1-", "0-3:0", "1;2"):
        assert _parse(lib, bad) is None, bad


def test_page_node_of_host_memory():
    """The placement check used on the GPU box: the node holding a page (this container has one
    node, or reports none)."""
    lib = _lib()
    buf = (ctypes.c_uint64 * 4096)()
    buf[0] = 1  # touched: the page exists
    node = lib.nhip_host_page_node(ctypes.addressof(buf))
    assert node in (-1, 0) or node >= 0


def _py_cpulist(text):
    """The kernel's cpulist syntax (lib/bitmap.c bitmap_parselist): "a", "a-b" or "a-b:stride"
    groups, separated by commas (the library also takes whitespace between groups); None when
    malformed."""
    import re
    out = set()
    for part in re.split(r"[,\s]+", text):
        if not part:
            continue
        rng, colon, stride = part.partition(":")
        a, dash, b = rng.partition("-")
        if not a.isdigit() or (dash and not b.isdigit()) or (colon and not stride.isdigit()):
            return None
        lo, hi = int(a), int(b) if dash else int(a)
        st = int(stride) if stride else 1
        if hi < lo or st <= 0 or hi > (1 << 20):
            return None
        out.update(range(lo, hi + 1, st))
    return sorted(out)


def test_cpulist_parse_matches_reference_grammar():
    """nhip_cpulist_parse on generated lists (single CPUs, ranges, strided ranges, overlaps, spaces)
    equals the grammar above; random byte strings never crash it and are either refused or parsed
    as the grammar parses them."""
    import random
    lib = _lib()
    rng = random.Random(0x5A)
    for _ in range(2000):
        parts = []
        for _ in range(rng.randint(1, 6)):
            a = rng.randint(0, 300)
            kind = rng.random()
            if kind < 0.4:
                parts.append(str(a))
            elif kind < 0.8:
                parts.append(f"{a}-{a + rng.randint(0, 64)}")
            else:
                parts.append(f"{a}-{a + rng.randint(0, 64)}:{rng.randint(1, 9)}")
        text = ",".join(parts) + rng.choice(["", "\n", " "])
        assert _parse(lib, text) == _py_cpulist(text), text
    alphabet = "0123456789,-: \nx"
    for _ in range(2000):
        text = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 24)))
        got, want = _parse(lib, text), _py_cpulist(text)
        assert got is None or got == want, text
