"""TCP / File / Hash / Prefix stores (SURVEY.md §4.3 'TCP store: set/get/wait/add, timeouts, multi-client')."""
import threading
import time
from datetime import timedelta

import pytest

from conftest import free_port


def C():
    import ringdp

    return ringdp._C


def test_tcpstore_basic_ops():
    m = C().TCPStore("127.0.0.1", 0, 1, True, 5000)
    m.set("a", b"1")
    m.set("s", "text")
    assert m.get("a") == b"1" and m.get("s") == b"text"
    assert m.add("cnt", 5) == 5 and m.add("cnt", -2) == 3
    assert m.get("cnt") == b"3"
    assert m.check(["a", "cnt"]) and not m.check(["a", "nope"])
    assert m.compare_set("cas", "", "x") == b"x"
    assert m.compare_set("cas", "wrong", "y") == b"x"
    assert m.compare_set("cas", "x", "y") == b"y"
    assert m.delete_key("a") and not m.delete_key("a")
    assert m.num_keys() >= 3


def test_tcpstore_multi_client_blocking_get():
    port = free_port()
    master = C().TCPStore("127.0.0.1", port, 3, True, 10000)
    clients = [C().TCPStore("127.0.0.1", port, 3, False, 10000) for _ in range(2)]
    got = []

    def reader(c):
        got.append(c.get("late"))

    ths = [threading.Thread(target=reader, args=(c,)) for c in clients]
    for t in ths:
        t.start()
    time.sleep(0.2)
    master.set("late", b"v")
    for t in ths:
        t.join(5)
    assert got == [b"v", b"v"]
    # add() is atomic across clients
    ths = [threading.Thread(target=lambda c=c: [c.add("n", 1) for _ in range(100)]) for c in clients]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert master.add("n", 0) == 200


def test_tcpstore_timeouts():
    m = C().TCPStore("127.0.0.1", 0, 1, True, 300)
    t0 = time.time()
    with pytest.raises(TimeoutError):
        m.get("missing")
    assert time.time() - t0 < 5
    with pytest.raises(TimeoutError):
        m.wait(["missing"], timedelta(milliseconds=200))
    m.set("x", b"1")
    m.wait(["x"])


def test_tcpstore_client_connect_timeout():
    port = free_port()
    t0 = time.time()
    with pytest.raises(TimeoutError):
        C().TCPStore("127.0.0.1", port, 2, False, 500)
    assert time.time() - t0 < 10


def test_filestore(tmp_path):
    p = str(tmp_path / "fs")
    a = C().FileStore(p, 2, 2000)
    b = C().FileStore(p, 2, 2000)
    a.set("k", b"v")
    assert b.get("k") == b"v"
    assert a.add("c", 2) == 2 and b.add("c", 3) == 5
    assert b.compare_set("k", "v", "w") == b"w"
    assert a.delete_key("k") and not b.check(["k"])
    with pytest.raises(TimeoutError):
        b.wait(["never"], timedelta(milliseconds=100))


def test_hash_and_prefix_store():
    h = C().HashStore(1000)
    p1 = C().PrefixStore("g1", h)
    p2 = C().PrefixStore("g2", h)
    p1.set("k", b"1")
    p2.set("k", b"2")
    assert p1.get("k") == b"1" and p2.get("k") == b"2"
    assert h.get("g1/k") == b"1"
    assert p1.add("n", 4) == 4 and h.get("g1/n") == b"4"


def test_pystore_adapter_over_torch_store():
    import torch.distributed as tdist

    ts = tdist.HashStore()
    ps = C().PyStore(ts, 2000)
    ps.set("a", b"b")
    assert ts.get("a") == b"b" and ps.get("a") == b"b"
    assert ps.add("n", 3) == 3
