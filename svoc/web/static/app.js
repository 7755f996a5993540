// svoc browser client: console + panels over the JSON API of svoc/web/app.py.
"use strict";

const $ = (id) => document.getElementById(id);
let eventCursor = 0;
let lastState = null;

function writeConsole(text, isUser = false) {
  const out = $("console-output");
  out.textContent += (isUser ? "> " : "") + text + "\n";
  out.scrollTop = out.scrollHeight;
}

async function send(cmd) {
  writeConsole(cmd, true);
  try {
    const r = await fetch("/api/query", {
      method: "POST", headers: {"Content-Type": "application/json"}, body: JSON.stringify({text: cmd}),
    });
    const j = await r.json();
    if (j.clear) $("console-output").textContent = "";
    else if (j.output) writeConsole(j.output);
  } catch (e) {
    writeConsole("request failed: " + e);
  }
  await refresh();
}

function median(xs) {
  const s = [...xs].sort((a, b) => a - b), n = s.length;
  return n % 2 ? s[(n - 1) / 2] : 0.5 * (s[n / 2 - 1] + s[n / 2]);
}

// the n_failing oracles farthest (sum of squared deviations) from the component-wise median
function flaggedOracles(preds, nFailing) {
  if (!preds || !preds.length) return new Set();
  const D = preds[0].length;
  const med = Array.from({length: D}, (_, d) => median(preds.map((p) => p[d])));
  const risk = preds.map((p, i) => [p.reduce((s, x, d) => s + (x - med[d]) ** 2, 0), i]);
  risk.sort((a, b) => b[0] - a[0] || b[1] - a[1]);
  return new Set(risk.slice(0, nFailing).map((r) => r[1]));
}

function svgEl(tag, attrs) {
  const e = document.createElementNS("http://www.w3.org/2000/svg", tag);
  for (const [k, v] of Object.entries(attrs)) e.setAttribute(k, v);
  return e;
}

function drawComponents(st) {
  const box = $("components");
  box.textContent = "";
  const preds = st.predictions;
  const flagged = flaggedOracles(preds, st.n_failing);
  for (let d = 0; d < st.dimension; ++d) {
    const div = document.createElement("div");
    div.className = "component";
    const name = document.createElement("div");
    name.className = "name";
    const svg = svgEl("svg", {viewBox: "0 0 300 70", preserveAspectRatio: "none"});
    const X = (v) => 10 + 280 * Math.min(1, Math.max(0, v));
    svg.appendChild(svgEl("line", {x1: 10, x2: 290, y1: 50, y2: 50, stroke: "#3b4656"}));
    for (const t of [0, 0.5, 1]) {
      const tx = svgEl("text", {x: X(t), y: 66, fill: "#7b8794", "font-size": 9, "text-anchor": "middle"});
      tx.textContent = t.toFixed(1);
      svg.appendChild(tx);
    }
    let label = st.labels[d];
    if (preds && preds.length) {
      const xs = preds.map((p) => p[d]);
      const mean = xs.reduce((a, b) => a + b, 0) / xs.length, med = median(xs);
      svg.appendChild(svgEl("line", {x1: X(mean), x2: X(mean), y1: 8, y2: 52, stroke: "#ebcb8b", "stroke-width": 2}));
      svg.appendChild(svgEl("line", {x1: X(med), x2: X(med), y1: 8, y2: 52, stroke: "#a3be8c", "stroke-width": 2}));
      xs.forEach((x, i) => {
        svg.appendChild(svgEl("circle", {cx: X(x), cy: 30 + ((i % 3) - 1) * 9, r: 5,
                                         fill: flagged.has(i) ? "#e0787a" : "#5fb3b3"}));
      });
      label += `  mean ${mean.toFixed(3)}  median ${med.toFixed(3)}`;
    }
    if (st.consensus_active && st.consensus.length > d) {
      const c = st.consensus[d];
      svg.appendChild(svgEl("line", {x1: X(c), x2: X(c), y1: 4, y2: 56, stroke: "#fff", "stroke-dasharray": "3 2"}));
      label += `  consensus ${c.toFixed(3)}`;
    }
    name.textContent = label;
    div.appendChild(name);
    div.appendChild(svg);
    box.appendChild(div);
  }
}

function fillSelect(sel, items, keep = true) {
  const prev = sel.value;
  sel.textContent = "";
  items.forEach((txt, i) => {
    const o = document.createElement("option");
    o.value = String(i);
    o.textContent = `${i}: ${txt}`;
    sel.appendChild(o);
  });
  if (keep && prev && Number(prev) < items.length) sel.value = prev;
}

function render(st) {
  lastState = st;
  $("engine-info").textContent = `engine: ${st.mode} mode on ${st.device} · window position ${st.position}`;
  st.reliability.forEach((r, i) => {
    const pct = st.consensus_active ? Math.round(Math.max(0, Math.min(1, r)) * 100) : 0;
    $(`bar-${i}`).style.width = pct + "%";
    $(`bar-text-${i}`).textContent = st.consensus_active ? r.toFixed(3) : "–";
  });
  const fmt = (xs) => xs.map((x) => x.toFixed(3)).join(", ");
  $("resume").textContent = `consensus_active: ${st.consensus_active}\n` +
    `consensus: ${fmt(st.consensus)}\nskewness: ${fmt(st.skewness)}\nkurtosis: ${fmt(st.kurtosis)}`;
  $("toggle-auto").textContent = st.flags.auto_fetch ? "auto_fetch off" : "auto_fetch on";
  drawComponents(st);
  fillSelect($("prop-caller"), st.admins);
  fillSelect($("vote-caller"), st.admins);
  fillSelect($("vote-which"), st.admins);
  fillSelect($("prop-old"), st.oracles);
  const open = st.propositions.map((p, i) => p ? `admin ${i}: oracle ${p.old_oracle} -> ${p.new_oracle}` : null)
    .filter((x) => x);
  $("propositions").textContent = open.length ? open.join("\n") : "no open proposition";
}

async function refresh() {
  try {
    const r = await fetch("/api/state");
    render(await r.json());
  } catch (e) { /* server gone: keep the last view */ }
}

async function pollEvents() {
  try {
    const r = await fetch(`/api/events?since=${eventCursor}`);
    const j = await r.json();
    j.lines.forEach((l) => writeConsole(l));
    if (j.lines.length) await refresh();
    eventCursor = j.next;
  } catch (e) { /* retry on the next tick */ }
}

$("console-form").addEventListener("submit", (ev) => {
  ev.preventDefault();
  const inp = $("console-input"), cmd = inp.value.trim();
  inp.value = "";
  if (cmd) send(cmd);
});
document.querySelectorAll("button[data-cmd]").forEach((b) => b.addEventListener("click", () => send(b.dataset.cmd)));
$("toggle-auto").addEventListener("click", () => send(lastState && lastState.flags.auto_fetch ? "auto_fetch off" : "auto_fetch on"));
$("propose-form").addEventListener("submit", (ev) => {
  ev.preventDefault();
  const addr = $("prop-new").value.trim();
  if (!addr.startsWith("0x")) { writeConsole("new address must start with 0x"); return; }
  send(`update_proposition ${$("prop-caller").value} ${$("prop-old").value} ${addr}`);
});
$("prop-clear").addEventListener("click", () => send(`update_proposition ${$("prop-caller").value} None`));
$("vote-form").addEventListener("submit", (ev) => {
  ev.preventDefault();
  send(`vote_for_a_proposition ${$("vote-caller").value} ${$("vote-which").value} yes`);
});
$("vote-no").addEventListener("click", () => send(`vote_for_a_proposition ${$("vote-caller").value} ${$("vote-which").value} no`));

writeConsole("type help for the command list");
refresh();
setInterval(pollEvents, 1500);
