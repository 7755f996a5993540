"""Browser UI (svoc/web/app.py vs client/web_interface.py + client/web/*): the page and its assets are
served, the console runs the CLI's commands, the panels' state follows the engine, the replacement
menu's commands reach governance, and auto-fetch output reaches the page through the event log."""
import time

import pytest
import torch

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from svoc.cli import Client  # noqa: E402
from svoc.web.app import EventLog, create_app  # noqa: E402


@pytest.fixture
def web(tmp_path):
    events = EventLog()
    cl = Client(db_path=str(tmp_path / "db.sqlite"), refresh_rate=0.05, emit=events.emit)
    with TestClient(create_app(cl, events)) as tc:
        yield tc, cl
    cl.close()


def q(tc, text):
    r = tc.post("/api/query", json={"text": text})
    assert r.status_code == 200
    return r.json()


def test_page_and_assets(web):
    tc, _ = web
    r = tc.get("/")
    assert r.status_code == 200 and "console-input" in r.text and "/static/app.js" in r.text
    for asset in ("app.js", "styles.css"):
        assert tc.get(f"/static/{asset}").status_code == 200


def test_console_round_trip_and_state(web):
    tc, cl = web
    assert "Commands" in q(tc, "help")["output"]
    assert q(tc, "clear")["clear"] is True
    st = tc.get("/api/state").json()
    assert st["consensus_active"] is False and st["predictions"] is None
    assert len(st["admins"]) == 3 and len(st["oracles"]) == 7 and st["dimension"] == 6
    out = q(tc, "fetch")["output"]
    assert "fetched" in out
    st = tc.get("/api/state").json()
    assert len(st["predictions"]) == 7 and len(st["predictions"][0]) == 6
    # the random-init encoder can give a column of equal values -> the contract reverts the 7th
    # update (zero variance); commit predictions with spread instead
    g = torch.Generator().manual_seed(3)
    cl.predictions = 0.1 + 0.8 * torch.rand(7, 6, generator=g)
    assert "REVERT" not in q(tc, "commit")["output"]
    st = tc.get("/api/state").json()
    assert st["consensus_active"] is True
    assert all(0.0 <= r <= 1.0 for r in st["reliability"])
    assert len(st["consensus"]) == 6
    assert "unknown command" in q(tc, "no_such_command")["output"]


def test_replacement_menu_commands(web):
    tc, cl = web
    st = tc.get("/api/state").json()
    assert st["propositions"] == [None, None, None]
    new = "0x1234abcd"
    q(tc, f"update_proposition 0 3 {new}")
    st = tc.get("/api/state").json()
    assert st["propositions"][0] == {"old_oracle": 3, "new_oracle": new}
    out = q(tc, "vote_for_a_proposition 1 0 yes")["output"]   # majority 2 of 3: applied
    assert "replaced" in out
    st = tc.get("/api/state").json()
    assert st["oracles"][3] == new
    q(tc, "update_proposition 2 None")
    assert tc.get("/api/state").json()["propositions"][2] is None


def test_auto_fetch_lines_reach_the_page(web):
    tc, cl = web
    assert "ENABLED" in q(tc, "auto_fetch on")["output"]
    lines, cursor, t0 = [], 0, time.time()
    while len(lines) < 2 and time.time() - t0 < 60:
        j = tc.get(f"/api/events?since={cursor}").json()
        lines += j["lines"]
        cursor = j["next"]
        time.sleep(0.05)
    assert "DISABLE" in q(tc, "auto_fetch off")["output"]
    assert len(lines) >= 2 and all("fetched" in l for l in lines)
    assert tc.get(f"/api/events?since={cursor}").json()["next"] >= cursor


def test_event_log_window():
    ev = EventLog(keep=3)
    for i in range(5):
        ev.emit(str(i))
    lines, nxt = ev.since(0)
    assert lines == ["2", "3", "4"] and nxt == 5
    assert ev.since(4) == (["4"], 5)
    assert ev.since(5) == ([], 5)
