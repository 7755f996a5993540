"""Command router: the reference client's text commands, driving the local engine instead of Sepolia.

The reference UI sends text commands to ``web_interface.query`` (client/web_interface.py:133-303,
help text :14-55).  Every command is kept; ``(S)`` commands that used to be Starknet RPC calls or
transactions now call the in-process consensus engine (one contract instance, exact wsad mode by
default, so the numbers are the contract's).  ``scraper on`` scrapes ``scraper_source`` (a URL or a
saved page, svoc/models/scraper.py) into the SQLite corpus on every fetch, or appends synthetic
comments when no source is set (no network on the GPU boxes); ``live_mode on`` classifies the newest
window.

Admin / oracle arguments accept an index or a ``0x...`` address; unlike the reference
(client/contract.py:95-123, survey §2.8-10) addresses are compared as integers, so both work.

    python -m svoc                     # interactive prompt
    python -m svoc -c "fetch" -c "commit" -c "resume"
"""
from __future__ import annotations

import os
import tempfile
import threading
from typing import Callable, Dict, List, Optional

import torch

from . import codec
from .api import OracleConsensus
from .models import corpus
from .models.encoder import ORACLE_LABELS, EncoderConfig
from .status import ConsensusRevert

HELP = """
Commands :
    - help / clear / exit
    - fetch
    - auto_fetch on/off (default: off)
    - auto_commit on/off (default: off, ie. fetch => commit)
    - auto_resume on/off (default: off, ie. commit => resume)
    - scraper on/off (default: off)       [scrape --scraper-source (or synthetic comments) on fetch]
    - live_mode on/off (default: off)     [classify the newest window]
    - contract_declaration_address
    - contract_address
    - (S) commit (call update_prediction for each oracle)
    - (S) resume
    - (S) consensus
    - (S) reliability_first_pass
    - (S) reliability
    - (S) is_consensus_active
    - (S) admin_list
    - (S) oracle_list
    - (S) dimension
    - (S) replacement_menu
    - (S) replacement_propositions
    - (S) update_proposition <caller_admin> None
    - (S) update_proposition <caller_admin> <old_oracle> <new_oracle>
    - (S) vote_for_a_proposition <caller_admin> <which_admin> yes/no
    - save <path> / load <path>           [.svoc checkpoint of the engine state]
    - report <path>                       [static HTML: scatter per label pair, reliability bars]
For <admin> <oracle> arguments, you can either specify the index or the address starting with "0x".
(S) = the consensus engine (the reference's Sepolia contract).
"""

N_ORACLES, N_FAILING, DIMENSION = 7, 2, 6        # client/common.py:8-9, 31
SIMULATION_REFRESH_RATE = 5.0                      # seconds between auto fetches (client/common.py:11)


class Client:
    def __init__(self, device: str = "cpu", mode: str = "exact", db_path: Optional[str] = None,
                 encoder: str = "tiny", dimension: int = DIMENSION, seed: int = 0,
                 refresh_rate: float = SIMULATION_REFRESH_RATE, emit: Callable[[str], None] = print,
                 scraper_source: Optional[str] = None):
        self.device = device
        self.scraper_source = scraper_source
        self.refresh_rate = float(refresh_rate)
        self.emit = emit                      # where the auto-fetch loop writes (the reference's console)
        self._lock = threading.RLock()        # one command at a time: the prompt and the auto-fetch loop
        self._auto_stop = threading.Event()
        self._auto_thread: Optional[threading.Thread] = None
        self._auto_lock = threading.Lock()     # serialises auto_fetch on/off (FastAPI runs handlers in threads)
        self.auto_fetches = 0
        self.admins = [codec.shortstring(x) for x in ("Akashi", "Ozu", "Higuchi")]
        self.oracles = [codec.shortstring(f"oracle_{i:02d}") for i in range(N_ORACLES)]
        self.contract = OracleConsensus(self.admins, True, 2, N_FAILING, True, 0, dimension, self.oracles,
                                        device=device, mode=mode)
        self.dimension = dimension
        self.db_path = db_path or os.path.join(tempfile.mkdtemp(prefix="svoc_"), "db.sqlite")
        self.conn = corpus.init_db(self.db_path)
        if corpus.get_last_comment_time(self.conn) is None:
            corpus.save_to_db(self.conn, corpus.synthetic_comments(200, seed))
        self.enc_cfg = EncoderConfig.tiny() if encoder == "tiny" else EncoderConfig()
        self._pipe = None
        self.position = 0
        self.predictions: Optional[torch.Tensor] = None
        self.flags = dict(auto_fetch=False, auto_commit=False, auto_resume=False, scraper=False, live_mode=False)
        self.seed = seed
        self.out: List[str] = []

    # ---- helpers -------------------------------------------------------------------------------
    def _pipeline(self):
        if self._pipe is None:
            from .config import ConsensusConfig
            from .engine import ConsensusEngine
            from .models.sentiment_oracle import SentimentOraclePipeline
            cfg = ConsensusConfig(n_oracles=N_ORACLES, dimension=6, n_failing_oracles=N_FAILING)
            # fp32 storage (reference resolution) on the CPU and on the GPU (consensus_fast_f32.hip)
            scratch = ConsensusEngine(cfg, 1, device=self.device, mode="fast", storage="fp32")
            self._pipe = SentimentOraclePipeline(scratch, enc_cfg=self.enc_cfg, seed=self.seed)
        return self._pipe

    def _admin(self, tok: str) -> int:
        return int(tok, 16) if tok.startswith("0x") else self.admins[int(tok)]

    def _oracle(self, tok: str) -> int:
        return int(tok, 16) if tok.startswith("0x") else self.contract.get_oracle_list()[int(tok)]

    def _fmt(self, felts) -> str:
        return "[" + ", ".join(codec.wsad_to_string(codec.felt_to_i128(f), 3) for f in felts) + "]"

    # ---- commands ------------------------------------------------------------------------------
    def fetch(self) -> str:
        """simulation_fetch (oracle_scheduler.py:155-161) + show_predictions (:136-153)."""
        if self.flags["scraper"]:
            if self.scraper_source:
                from .models.scraper import scrape_once
                scrape_once(self.conn, self.scraper_source)
            else:
                corpus.save_to_db(self.conn, corpus.synthetic_comments(30, seed=self.position + 1))
        comments, stamps, self.position = corpus.read_window_from_db(self.conn, self.position)
        if self.flags["live_mode"]:
            n = self.conn.execute("SELECT COUNT(id) FROM comments").fetchone()[0]
            comments, stamps, _ = corpus.read_window_from_db(self.conn, max(0, n - corpus.WINDOW_SIZE - 50))
        p = self._pipeline()
        vocab = p.encoder.cfg.vocab_size
        ids, mask = corpus.tokenize(comments, seq_len=min(128, p.encoder.cfg.max_positions - 2), vocab=vocab)
        dev = p.engine.device
        scores = p.classify(ids.to(dev), mask.to(dev))
        self.predictions = p.oracles(scores, seed=self.seed * 7919 + self.position)[0].cpu()
        from .utils.diagnostics import show_predictions
        s = f"fetched {len(comments)} comments from {stamps[-1] if stamps else '-'} UTC\n"
        s += show_predictions(self.predictions, N_FAILING, ORACLE_LABELS)
        if self.flags["auto_commit"]:
            s += "\n" + self.commit()
        return s

    # ---- auto fetch (simulation_mode, client/oracle_scheduler.py:163-171) -------------------------
    def _auto_fetch_loop(self, stop: threading.Event) -> None:
        """Fetch, then sleep refresh_rate seconds, until ``stop`` is set.  The reference runs this loop
        inside the UI handler with eel.sleep; here it is a daemon thread next to the prompt.  Every loop
        owns its stop event, so a loop that was switched off never comes back to life."""
        while not stop.is_set():
            with self._lock:
                if stop.is_set() or not self.flags["auto_fetch"]:
                    break
                try:
                    out = self.fetch()
                except Exception as e:   # a failed fetch is reported, the loop keeps its period
                    out = f"auto_fetch error: {e!r}"
                self.auto_fetches += 1
            self.emit(out)
            stop.wait(self.refresh_rate)

    def set_auto_fetch(self, on: bool) -> str:
        with self._auto_lock:
            self.flags["auto_fetch"] = bool(on)
            t = self._auto_thread
            if on:
                if t is not None and t.is_alive() and not self._auto_stop.is_set():
                    return "Auto-Fetch: ENABLED"      # already running: never a second loop
                # (a loop switched off but still finishing a fetch exits on its own, already set event)
                self._auto_stop = threading.Event()
                self._auto_thread = threading.Thread(target=self._auto_fetch_loop, args=(self._auto_stop,),
                                                     name="svoc-auto-fetch", daemon=True)
                self._auto_thread.start()
                return "Auto-Fetch: ENABLED"
            self._auto_stop.set()
            self._auto_thread = None
        if t is not None and t is not threading.current_thread():
            t.join(timeout=max(1.0, 2 * self.refresh_rate) + 60.0)
        return "Auto-Fetch: DISABLE"

    def close(self) -> None:
        self.set_auto_fetch(False)

    def commit(self) -> str:
        """update_all_the_predictions (client/contract.py:200-208): one update per oracle, in order."""
        if self.predictions is None:
            return "nothing to commit: run fetch first"
        lines = []
        for o, pred in zip(self.contract.get_oracle_list(), self.predictions.tolist()):
            felts = [codec.float_to_fwsad(x) for x in pred[: self.dimension]]
            try:
                st = self.contract.update_prediction(o, felts)
                lines.append(f"oracle {hex(o)}: {st.name}")
            except ConsensusRevert as e:
                lines.append(f"oracle {hex(o)}: REVERT {e.status.name}")
        if self.flags["auto_resume"]:
            lines.append(self.resume())
        return "\n".join(lines)

    def resume(self) -> str:
        c = self.contract
        s = [f"consensus_active: {c.consensus_active()}",
             f"consensus: {self._fmt(c.get_consensus_value())}",
             f"reliability first pass: {codec.fwsad_to_float(c.get_first_pass_consensus_reliability()):.3f}",
             f"reliability second pass: {codec.fwsad_to_float(c.get_second_pass_consensus_reliability()):.3f}",
             f"skewness: {self._fmt(c.get_skewness())}",
             f"kurtosis: {self._fmt(c.get_kurtosis())}"]
        return "\n".join(s)

    def query(self, text: str) -> str:
        sp = text.split()
        if sp and sp[0] == "auto_fetch" and len(sp) == 2:   # outside the lock: it may join the loop
            return self.set_auto_fetch(sp[1] == "on")
        with self._lock:
            return self._query(text)

    def _query(self, text: str) -> str:
        sp = text.split()
        if not sp:
            return ""
        cmd, args = sp[0], sp[1:]
        c = self.contract
        onoff = lambda k: self.flags.__setitem__(k, args[0] == "on") or f"{k}: {self.flags[k]}"  # noqa: E731
        simple: Dict[str, Callable[[], str]] = {
            "help": lambda: HELP,
            "clear": lambda: "",
            "fetch": self.fetch,
            "commit": self.commit,
            "resume": self.resume,
            "consensus": lambda: self._fmt(c.get_consensus_value()),
            "reliability_first_pass": lambda: f"{codec.fwsad_to_float(c.get_first_pass_consensus_reliability()):.6f}",
            "reliability": lambda: f"{codec.fwsad_to_float(c.get_second_pass_consensus_reliability()):.6f}",
            "is_consensus_active": lambda: str(c.consensus_active()),
            "admin_list": lambda: "\n".join(hex(a) for a in c.get_admin_list()),
            "oracle_list": lambda: "\n".join(hex(a) for a in c.get_oracle_list()),
            "dimension": lambda: str(c.get_predictions_dimension()),
            "replacement_propositions": lambda: str(c.get_replacement_propositions()),
            "replacement_menu": lambda: "\n".join(
                f"admin {i} ({hex(a)}): {p}" for i, (a, p) in
                enumerate(zip(c.get_admin_list(), c.get_replacement_propositions()))),
            "contract_declaration_address": lambda: "local engine (no declaration: not on chain)",
            "contract_address": lambda: f"local engine, mode={c.engine.mode}, device={c.engine.device}",
        }
        try:
            if cmd in simple:
                return simple[cmd]()
            if cmd in ("auto_commit", "auto_resume", "scraper", "live_mode") and args:
                return onoff(cmd)
            if cmd == "update_proposition" and len(args) in (2, 3):
                caller = self._admin(args[0])
                prop = None if args[1] == "None" else (
                    int(args[1]) if not args[1].startswith("0x") else c.get_oracle_list().index(int(args[1], 16)),
                    int(args[2], 16) if args[2].startswith("0x") else int(args[2]))
                c.update_proposition(caller, prop)
                return "proposition updated"
            if cmd == "vote_for_a_proposition" and len(args) == 3:
                caller = self._admin(args[0])
                which = int(args[1]) if not args[1].startswith("0x") else c.get_admin_list().index(int(args[1], 16))
                ok = args[2].upper() == "YES"
                if args[2].upper() not in ("YES", "NO"):
                    return "usage: vote_for_a_proposition <caller_admin> <which_admin> yes/no"
                applied = c.vote_for_a_proposition(caller, which, ok)
                return "vote recorded" + (" -> oracle replaced" if applied else "")
            if cmd == "report" and args:
                from .utils.report import write_report
                labels = ORACLE_LABELS[: self.dimension] if self.dimension <= len(ORACLE_LABELS) else None
                write_report(args[0], c.engine, [0], labels, c.get_oracle_list())
                return f"report written to {args[0]}"
            if cmd in ("save", "load") and args:
                from . import state
                if cmd == "save":
                    state.save(c._svc, args[0])
                    return f"saved {args[0]}"
                c._svc = state.load(args[0], device=self.device)
                return f"loaded {args[0]}"
        except ConsensusRevert as e:
            return f"REVERT: {e.status.name}"
        except (ValueError, IndexError) as e:
            return f"error: {e}"
        return f"unknown command: {text!r} (try help)"
