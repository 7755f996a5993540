"""Command router (client/web_interface.py:133-303 equivalents) on the local exact engine."""
import pytest

from svoc import ops as svops
from svoc.cli import Client

pytestmark = pytest.mark.skipif(not svops.available(), reason="svoc/_C.so not built")


def test_fetch_commit_resume_governance(tmp_path):
    cl = Client(device="cpu", mode="exact", db_path=str(tmp_path / "db.sqlite"), seed=1)
    assert "optimism" in cl.query("fetch")
    out = cl.query("commit")
    assert out.count("NOT_ACTIVE") == 6 and "OK" in out.splitlines()[-1]
    assert cl.query("is_consensus_active") == "True"
    r = float(cl.query("reliability"))
    assert 0.0 <= r <= 1.0
    assert len(cl.query("oracle_list").splitlines()) == 7
    assert cl.query("dimension") == "6"
    assert cl.query("update_proposition 0 6 0x1234") == "proposition updated"
    assert cl.query("vote_for_a_proposition 0 0 yes") == "vote recorded"
    assert "replaced" in cl.query("vote_for_a_proposition 1 0 yes")
    assert cl.query("oracle_list").splitlines()[6] == "0x1234"
    assert cl.query("update_proposition 0 9 0x99").startswith("REVERT")
    assert cl.query("save " + str(tmp_path / "c.svoc")).startswith("saved")
    assert cl.query("load " + str(tmp_path / "c.svoc")).startswith("loaded")
    assert cl.query("oracle_list").splitlines()[6] == "0x1234"
    assert "unknown" in cl.query("frobnicate")
    assert "Commands" in cl.query("help")


def test_report_html(tmp_path):
    cl = Client(device="cpu", mode="exact", db_path=str(tmp_path / "db.sqlite"), seed=1)
    cl.query("fetch")
    cl.query("commit")
    out = tmp_path / "r.html"
    assert cl.query(f"report {out}").startswith("report written")
    doc = out.read_text()
    assert doc.count("<svg") == 3 and "reliability (second pass)" in doc and "optimism / anger" in doc


def test_auto_fetch_is_a_periodic_loop(tmp_path):
    """auto_fetch on: fetch, sleep refresh_rate, repeat while on (oracle_scheduler.py:163-171);
    auto_commit chains a commit after each fetch; off stops the loop."""
    import time
    outs = []
    cl = Client(db_path=str(tmp_path / "db.sqlite"), refresh_rate=0.05, emit=outs.append)
    cl.query("auto_commit on")
    assert cl.query("auto_fetch on") == "Auto-Fetch: ENABLED"
    t0 = time.time()
    while cl.auto_fetches < 3 and time.time() - t0 < 120:
        time.sleep(0.02)
    assert cl.query("auto_fetch off") == "Auto-Fetch: DISABLE"
    n = cl.auto_fetches
    assert n >= 3 and len(outs) >= 3 and all("fetched" in o for o in outs)
    assert any("oracle 0x" in o for o in outs)          # auto_commit ran
    time.sleep(0.2)
    assert cl.auto_fetches == n                          # stopped


def test_auto_fetch_concurrent_toggles_keep_one_loop(tmp_path):
    """Concurrent 'auto_fetch on' requests (FastAPI handlers run in a thread pool) start one loop; 'on'
    right after 'off' never revives the old loop next to the new one."""
    import threading
    import time
    cl = Client(db_path=str(tmp_path / "db.sqlite"), refresh_rate=0.05, emit=lambda s: None)
    ts = [threading.Thread(target=cl.set_auto_fetch, args=(True,)) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    loops = [t for t in threading.enumerate() if t.name == "svoc-auto-fetch"]
    assert len(loops) == 1
    for _ in range(3):
        cl.set_auto_fetch(False)
        cl.set_auto_fetch(True)
    time.sleep(0.3)
    assert len([t for t in threading.enumerate() if t.name == "svoc-auto-fetch" and t.is_alive()]) == 1
    cl.set_auto_fetch(False)
    time.sleep(0.2)
    assert not [t for t in threading.enumerate() if t.name == "svoc-auto-fetch" and t.is_alive()]
