"""Browser UI for the client (client/web_interface.py:61-303, client/web/*).

The reference serves ``client/web`` through Eel and calls Python from JavaScript (``query(text)``)
and JavaScript from Python (``writeToConsole``, ``updateProgressBar``, ``setSepoliaConsole``,
``updateComponents``, ``refreshReplacementMenu``).  Here a FastAPI app serves the page and the
JavaScript polls three JSON endpoints; every command still goes through the same text router
(``svoc.cli.Client.query``), so the console accepts exactly the CLI's commands.

    GET  /                 the page (svoc/web/static/index.html)
    POST /api/query        {"text": "..."} -> {"output": "...", "clear": bool}
    GET  /api/state        engine outputs + last fetched predictions + governance, for the panels
    GET  /api/events?since=k   console lines emitted by the auto-fetch loop since line k

    python -m svoc.web --port 8080 [--device cuda] [--mode fast]
"""
from __future__ import annotations

import argparse
import os
import threading
from typing import List, Optional

from .. import codec
from ..cli import DIMENSION, N_FAILING, Client
from ..models.encoder import ORACLE_LABELS
from ..status import ConsensusRevert

STATIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static")


class EventLog:
    """Lines the auto-fetch loop writes (the reference's ``eel.writeToConsole`` from the scheduler),
    numbered so a poller can ask for what it has not seen."""

    def __init__(self, keep: int = 1000):
        self.keep = keep
        self._lines: List[str] = []
        self._first = 0
        self._lock = threading.Lock()

    def emit(self, text: str) -> None:
        with self._lock:
            self._lines.append(text)
            if len(self._lines) > self.keep:
                drop = len(self._lines) - self.keep
                del self._lines[:drop]
                self._first += drop

    def since(self, k: int):
        with self._lock:
            start = max(k, self._first) - self._first
            return self._lines[start:], self._first + len(self._lines)


def _floats(felts) -> List[float]:
    return [codec.fwsad_to_float(f) for f in felts]


def state_dict(cl: Client) -> dict:
    """Everything the panels draw: the resume block, the two reliability bars, the per-component
    oracle plot (predictions of the last fetch, their mean and median, the engine consensus) and the
    replacement menu (admins, oracles, open propositions)."""
    c = cl.contract
    with cl._lock:
        preds = None if cl.predictions is None else cl.predictions[:, : cl.dimension].tolist()
        try:
            props = c.get_replacement_propositions()
        except ConsensusRevert:
            props = []
        oracles = c.get_oracle_list()
        labels = ORACLE_LABELS[: cl.dimension] if cl.dimension <= len(ORACLE_LABELS) else \
            [f"dim {i}" for i in range(cl.dimension)]
        return dict(
            dimension=cl.dimension,
            n_failing=N_FAILING,
            labels=labels,
            consensus_active=c.consensus_active(),
            consensus=_floats(c.get_consensus_value()),
            reliability=[codec.fwsad_to_float(c.get_first_pass_consensus_reliability()),
                         codec.fwsad_to_float(c.get_second_pass_consensus_reliability())],
            skewness=_floats(c.get_skewness()),
            kurtosis=_floats(c.get_kurtosis()),
            predictions=preds,
            admins=[hex(a) for a in c.get_admin_list()],
            oracles=[hex(a) for a in oracles],
            propositions=[None if p is None else dict(old_oracle=int(p[0]), new_oracle=hex(int(p[1])))
                          for p in props],
            flags=dict(cl.flags),
            position=cl.position,
            mode=c.engine.mode,
            device=str(c.engine.device),
        )


def create_app(client: Optional[Client] = None, events: Optional[EventLog] = None):
    import contextlib

    from fastapi import Body, FastAPI
    from fastapi.responses import FileResponse, JSONResponse
    from fastapi.staticfiles import StaticFiles

    events = events or EventLog()
    cl = client or Client(emit=events.emit)
    if client is not None:
        client.emit = events.emit

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        yield
        cl.close()   # stops the auto-fetch thread

    app = FastAPI(title="svoc client", lifespan=lifespan)
    app.state.client, app.state.events = cl, events
    app.mount("/static", StaticFiles(directory=STATIC), name="static")

    @app.get("/")
    def index():
        return FileResponse(os.path.join(STATIC, "index.html"))

    @app.post("/api/query")
    def query(text: str = Body(..., embed=True)):
        text = text.strip()
        if text == "exit":   # the page stays up; the server is stopped from its terminal
            return dict(output="exit: close the tab / stop the server", clear=False)
        out = cl.query(text)
        return dict(output=out, clear=text == "clear")

    @app.get("/api/state")
    def state():
        return JSONResponse(state_dict(cl))

    @app.get("/api/events")
    def poll(since: int = 0):
        lines, nxt = events.since(since)
        return dict(lines=lines, next=nxt)

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="svoc browser UI (client/web_interface.py)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--mode", default="exact", choices=["exact", "fast"])
    ap.add_argument("--db", default=None)
    ap.add_argument("--dimension", type=int, default=DIMENSION)
    ap.add_argument("--refresh", type=float, default=5.0)
    ap.add_argument("--scraper-source", default=None)
    ap.add_argument("--disable_startup_fetch", action="store_true")
    a = ap.parse_args(argv)
    import uvicorn
    events = EventLog()
    cl = Client(device=a.device, mode=a.mode, db_path=a.db, dimension=a.dimension, refresh_rate=a.refresh,
                emit=events.emit, scraper_source=a.scraper_source)
    if not a.disable_startup_fetch:   # client/main.py: a first fetch at startup
        events.emit(cl.query("fetch"))
    uvicorn.run(create_app(cl, events), host=a.host, port=a.port, log_level="warning")
    return 0
