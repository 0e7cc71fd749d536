// tinychat: dependency-free chat UI for the xot ChatGPT-compatible API
// (feature parity with the reference UI, xotorch/tinychat/index.js: history in localStorage,
// streaming completions with client-side TTFT and tokens/s, model picker fed by /initial_models and
// the /modelpool SSE stream, download/delete, topology and download-progress panels).
"use strict";

const $ = (id) => document.getElementById(id);
const state = {
  histories: JSON.parse(localStorage.getItem("xot.histories") || "[]"),
  current: null,           // {id, title, model, messages: [{role, content}]}
  models: {},              // id -> {name, downloaded, download_percentage, ...}
  model: localStorage.getItem("xot.model") || null,
  abort: null,
};

function save() {
  localStorage.setItem("xot.histories", JSON.stringify(state.histories.slice(0, 100)));
  if (state.model) localStorage.setItem("xot.model", state.model);
}

function escapeHtml(s) {
  return s.replace(/[&<>"']/g, (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;" }[c]));
}

// minimal markdown: fenced code blocks and inline code; everything else is plain text
function render(text) {
  const parts = text.split(/```/);
  return parts.map((p, i) => {
    if (i % 2 === 1) {
      const nl = p.indexOf("\n");
      const body = nl >= 0 ? p.slice(nl + 1) : p;
      return `<pre><code>${escapeHtml(body)}</code></pre>`;
    }
    return escapeHtml(p).replace(/`([^`]+)`/g, "<code>$1</code>");
  }).join("");
}

function drawMessages() {
  const box = $("messages");
  box.innerHTML = "";
  const msgs = state.current ? state.current.messages : [];
  for (const m of msgs) {
    const d = document.createElement("div");
    d.className = `msg ${m.role}`;
    d.innerHTML = render(m.content);
    box.appendChild(d);
  }
  box.scrollTop = box.scrollHeight;
}

function drawHistory() {
  const ul = $("history");
  ul.innerHTML = "";
  for (const h of state.histories) {
    const li = document.createElement("li");
    li.className = state.current && h.id === state.current.id ? "active" : "";
    const t = document.createElement("span");
    t.textContent = h.title || "(untitled)";
    t.onclick = () => { state.current = h; drawHistory(); drawMessages(); };
    const x = document.createElement("button");
    x.textContent = "×";
    x.title = "Delete conversation";
    x.onclick = (e) => {
      e.stopPropagation();
      state.histories = state.histories.filter((o) => o.id !== h.id);
      if (state.current && state.current.id === h.id) state.current = null;
      save(); drawHistory(); drawMessages();
    };
    li.append(t, x);
    ul.appendChild(li);
  }
}

function newChat() {
  state.current = null;
  $("stats").textContent = "";
  drawHistory(); drawMessages();
}

// ------------------------------------------------------------------ models
function drawModels() {
  const sel = $("model-select");
  const prev = state.model;
  sel.innerHTML = "";
  for (const [id, m] of Object.entries(state.models)) {
    const o = document.createElement("option");
    o.value = id;
    let tag = "";
    if (m.downloaded) tag = " ✓";
    else if (m.download_percentage) tag = ` (${m.download_percentage.toFixed(0)}%)`;
    o.textContent = (m.name || id) + tag;
    sel.appendChild(o);
  }
  if (prev && state.models[prev]) sel.value = prev;
  state.model = sel.value;
  const m = state.models[state.model] || {};
  $("model-status").textContent = m.downloaded ? "downloaded" :
    (m.total_size ? `${fmtBytes(m.total_downloaded || 0)} / ${fmtBytes(m.total_size)}` : "");
}

function fmtBytes(n) {
  const u = ["B", "KB", "MB", "GB", "TB"];
  let i = 0;
  while (n >= 1024 && i < u.length - 1) { n /= 1024; i++; }
  return `${n.toFixed(1)} ${u[i]}`;
}

async function loadModels() {
  try {
    state.models = await (await fetch("/initial_models")).json();
    drawModels();
  } catch (e) { console.warn("initial_models", e); }
  // live status stream
  try {
    const es = new EventSource("/modelpool");
    es.onmessage = (ev) => {
      if (ev.data === "[DONE]") { es.close(); return; }
      const upd = JSON.parse(ev.data);
      for (const [id, info] of Object.entries(upd)) state.models[id] = { ...(state.models[id] || {}), ...info };
      drawModels();
    };
    es.onerror = () => es.close();
  } catch (e) { console.warn("modelpool", e); }
}

async function downloadModel() {
  const r = await fetch("/download", { method: "POST", headers: { "Content-Type": "application/json" },
                                       body: JSON.stringify({ model: state.model }) });
  const d = await r.json();
  $("model-status").textContent = d.message || d.error || d.detail || "";
}

async function deleteModel() {
  if (!confirm(`Delete the downloaded files of ${state.model}?`)) return;
  const r = await fetch(`/models/${encodeURIComponent(state.model)}`, { method: "DELETE" });
  const d = await r.json();
  $("model-status").textContent = d.message || d.detail || "";
  if (r.ok && state.models[state.model]) state.models[state.model].downloaded = false;
  drawModels();
}

// ------------------------------------------------------------------ chat
async function send(text) {
  if (!text.trim() || state.abort) return;
  if (!state.current) {
    state.current = { id: crypto.randomUUID ? crypto.randomUUID() : String(Date.now()), title: text.slice(0, 40),
                      model: state.model, messages: [] };
    state.histories.unshift(state.current);
  }
  const conv = state.current;
  conv.messages.push({ role: "user", content: text });
  const reply = { role: "assistant", content: "" };
  conv.messages.push(reply);
  drawHistory(); drawMessages();
  const ctrl = new AbortController();
  state.abort = ctrl;
  $("send").hidden = true; $("stop").hidden = false;
  const t0 = performance.now();
  let tFirst = null, nTok = 0;
  const body = {
    model: state.model, stream: true,
    messages: conv.messages.slice(0, -1).map(({ role, content }) => ({ role, content })),
    temperature: parseFloat($("temperature").value),
    max_tokens: parseInt($("max-tokens").value, 10),
  };
  try {
    const r = await fetch("/v1/chat/completions", { method: "POST", signal: ctrl.signal,
      headers: { "Content-Type": "application/json" }, body: JSON.stringify(body) });
    if (!r.ok) throw new Error((await r.json()).detail || r.statusText);
    const reader = r.body.getReader();
    const dec = new TextDecoder();
    let buf = "";
    for (;;) {
      const { value, done } = await reader.read();
      if (done) break;
      buf += dec.decode(value, { stream: true });
      let i;
      while ((i = buf.indexOf("\n\n")) >= 0) {
        const line = buf.slice(0, i).trim();
        buf = buf.slice(i + 2);
        if (!line.startsWith("data: ")) continue;
        const data = line.slice(6);
        if (data === "[DONE]") continue;
        const chunk = JSON.parse(data);
        const delta = chunk.choices && chunk.choices[0] && chunk.choices[0].delta;
        if (delta && delta.content) {
          if (tFirst === null) tFirst = performance.now();
          nTok += 1;  // one SSE chunk per sampled token group
          reply.content += delta.content;
          drawMessages();
          const dt = (performance.now() - tFirst) / 1000;
          $("stats").textContent = `TTFT ${((tFirst - t0) / 1000).toFixed(2)} s · ` +
            (dt > 0 ? `${(nTok / dt).toFixed(1)} tok/s` : "");
        }
      }
    }
  } catch (e) {
    if (e.name !== "AbortError") reply.content += `\n[error: ${e.message}]`;
  } finally {
    state.abort = null;
    $("send").hidden = false; $("stop").hidden = true;
    save(); drawMessages();
  }
}

// ------------------------------------------------------------------ ring / downloads panels
async function pollTopology() {
  try {
    const t = await (await fetch("/v1/topology")).json();
    const box = $("topology");
    box.innerHTML = "";
    const nodes = Object.entries(t.nodes || {});
    let tf = 0;
    for (const [id, c] of nodes) {
      tf += (c.flops && c.flops.fp16) || 0;
      const d = document.createElement("div");
      d.className = "peer" + (id === t.active_node_id ? " active" : "");
      d.textContent = `${id.slice(0, 12)} · ${c.chip} · ${(c.memory / 1024).toFixed(0)} GB`;
      box.appendChild(d);
    }
    const s = document.createElement("div");
    s.className = "muted";
    s.textContent = `${nodes.length} peer(s), ${tf.toFixed(0)} fp16 TFLOPS`;
    box.appendChild(s);
  } catch (e) { $("topology").textContent = "topology unavailable"; }
}

async function pollDownloads() {
  try {
    const p = await (await fetch("/v1/download/progress")).json();
    const box = $("downloads");
    box.innerHTML = "";
    for (const [node, d] of Object.entries(p)) {
      const pct = d.total_bytes ? (100 * d.downloaded_bytes) / d.total_bytes : 0;
      const row = document.createElement("div");
      row.innerHTML = `<div class="muted">${escapeHtml(node.slice(0, 12))} ${escapeHtml(String(d.repo_id || ""))} ` +
        `${pct.toFixed(1)}%</div><div class="bar"><div style="width:${pct}%"></div></div>`;
      box.appendChild(row);
    }
  } catch (e) { /* ignore */ }
}

// ------------------------------------------------------------------ wiring
window.addEventListener("DOMContentLoaded", () => {
  $("new-chat").onclick = newChat;
  $("model-select").onchange = (e) => { state.model = e.target.value; save(); drawModels(); };
  $("download-model").onclick = downloadModel;
  $("delete-model").onclick = deleteModel;
  $("stop").onclick = () => state.abort && state.abort.abort();
  $("composer").onsubmit = (e) => { e.preventDefault(); const v = $("prompt").value; $("prompt").value = ""; send(v); };
  $("prompt").addEventListener("keydown", (e) => {
    if (e.key === "Enter" && !e.shiftKey) { e.preventDefault(); $("composer").requestSubmit(); }
  });
  drawHistory(); drawMessages();
  loadModels();
  pollTopology(); setInterval(pollTopology, 5000);
  pollDownloads(); setInterval(pollDownloads, 1000);
});
