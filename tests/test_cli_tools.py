"""CLI parity (`shellac -s -c -p -t -z`), the ab-style load generator, profiling helper."""
import cProfile
import os
import socket
import subprocess
import sys
import time

import pytest

from shellac_amd.bench.ab import run as ab_run, write_gnuplot
from shellac_amd.server.proxy import Server, build_arg_parser, main, parse_server_list
from shellac_amd.utils.fakemc import FakeMemcached
from shellac_amd.utils.httpclient import HttpClient
from shellac_amd.utils.origin import Origin

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_argparse_reference_flags():
    a = build_arg_parser().parse_args(["-s", "a:81,b", "-c", "m1,m2:11212", "-p", "9090", "-t", "60", "-z"])
    assert (a.servers, a.caches, a.port, a.ttl, a.compress) == ("a:81,b", "m1,m2:11212", 9090, 60, True)
    assert parse_server_list("127.0.0.1:81,localhost", 80) == [("127.0.0.1", 81), ("127.0.0.1", 80)]
    g = build_arg_parser().parse_args(["-s", "a", "--cache", "hbm", "--no-hbm-filter",
                                       "--hbm-spin-us", "0"])
    assert (g.cache, g.no_hbm_filter, g.hbm_spin_us) == ("hbm", True, 0)
    assert build_arg_parser().parse_args(["-s", "a"]).no_hbm_filter is False


def test_missing_servers_exits_1(capsys):
    assert main([]) == 1
    assert "No upstream web servers specified" in capsys.readouterr().out


def test_cli_end_to_end_with_memcached_and_kill():
    o = Origin().start()
    f = FakeMemcached().start()
    port = free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "shellac_amd", "-s", f"127.0.0.1:{o.port}",
                          "-c", f"127.0.0.1:{f.port}", "-p", str(port), "-t", "30"],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, cwd=ROOT)
    try:
        deadline = time.time() + 60
        c = None
        while time.time() < deadline:
            try:
                c = HttpClient(port=port, timeout=5)
                break
            except OSError:
                time.sleep(0.2)
        assert c is not None, p.stdout.read().decode()
        assert c.get("/cli").status() == 200
        time.sleep(0.2)
        assert c.get("/cli").status() == 200
        assert o.hits["/cli"] == 1 and len(f.data) == 1
        c.send(HttpClient.request_bytes("/kill"))
        assert p.wait(timeout=20) == 0
        assert b"Running Shellac on port" in p.stdout.read()
    finally:
        if p.poll() is None:
            p.kill()
        o.stop()
        f.stop()


def test_loadgen_ab_equivalent(tmp_path):
    o = Origin(body_bytes=500).start()
    try:
        with Server([("127.0.0.1", o.port)], port=0, backend_kind="dram", dram_mb=32,
                    client_max_reqs=1 << 30) as px:
            url = f"http://127.0.0.1:{px.port}/ab.html"
            r = ab_run(url, requests=2000, concurrency=10, keepalive=True,
                       headers=["Accept-Encoding: gzip"], depth=2, threads=2)
            assert r["completed"] == 2000 and r["errors"] == 0 and r["non2xx"] == 0
            assert r["rps"] > 0 and r["latency_ms"]["p99"] >= r["latency_ms"]["p50"]
            assert o.hits["/ab.html"] == 1
            g = tmp_path / "shellac.dat"
            write_gnuplot(str(g), r, time.time())
            lines = g.read_text().splitlines()
            assert len(lines) == 2001 and lines[0].startswith("starttime")
            # the server closing connections (max requests) is handled like ab -k
            with Server([("127.0.0.1", o.port)], port=0, backend_kind="dram", dram_mb=32,
                        client_max_reqs=7) as px2:
                r2 = ab_run(f"http://127.0.0.1:{px2.port}/x", requests=300, concurrency=4)
                assert r2["completed"] == 300
    finally:
        o.stop()


def test_prof_helper(tmp_path, capsys):
    from shellac_amd.utils.prof import main as prof_main

    out = tmp_path / "out.prof"
    cProfile.runctx("sum(range(1000))", {}, {}, str(out))
    assert prof_main([str(out)]) == 0
    assert "cumulative" in capsys.readouterr().out


def test_cli_hot_spreading_flags():
    """`shellac` / `shellac-cached` take the HBM tier's hot-object spreading knobs (SURVEY.md
    §5.8): --hot-objects (0 = plain ketama) and --hot-refresh-ms."""
    from shellac_amd.server.proxy import build_arg_parser

    a = build_arg_parser().parse_args(["-s", "127.0.0.1:80", "--cache", "hbm",
                                       "--hot-objects", "0", "--hot-refresh-ms", "250"])
    assert a.hot_objects == 0 and a.hot_refresh_ms == 250
    a = build_arg_parser().parse_args(["-s", "127.0.0.1:80"])
    assert a.hot_objects == 1024 and a.hot_refresh_ms == 1000
