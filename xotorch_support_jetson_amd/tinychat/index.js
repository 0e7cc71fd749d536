// tinychat: dependency-free chat UI for the xot ChatGPT-compatible API
// (feature parity with the reference UI, xotorch/tinychat/index.js: history in localStorage, streaming
// completions with client-side TTFT and tokens/s, image attachments sent as image_url parts (:157-230), a
// pending message that survives a reload or a failed send and is resumed (:198, :476-479), markdown with
// highlighted fenced code (:732-740; here without marked / highlight.js), the model picker fed by
// /initial_models and the /modelpool SSE stream, download/delete, topology and download-progress panels).
"use strict";

// ------------------------------------------------------------------ pure helpers (also run under node: tests)
function escapeHtml(s) {
  return String(s).replace(/[&<>"']/g, (c) => ({ "&": "&amp;", "<": "&lt;", ">": "&gt;", '"': "&quot;", "'": "&#39;" }[c]));
}

const KEYWORDS = {
  python: "and as assert async await break class continue def del elif else except False finally for from global if import in is lambda None nonlocal not or pass raise return True try while with yield",
  js: "async await break case catch class const continue default delete do else export extends false finally for function if import in instanceof let new null of return static super switch this throw true try typeof undefined var void while yield",
  c: "auto bool break case char class const constexpr continue default delete do double else enum extern false float for if inline int long namespace new nullptr private public return short signed sizeof static struct switch template this true typedef typename union unsigned using virtual void volatile while __global__ __device__ __shared__",
  shell: "case do done elif else esac export fi for function if in local return then until while",
};
const LANG_ALIASES = { py: "python", python: "python", javascript: "js", js: "js", ts: "js", typescript: "js", json: "js",
                       c: "c", cpp: "c", "c++": "c", cc: "c", h: "c", hip: "c", cuda: "c", rust: "c", go: "c", java: "c",
                       sh: "shell", bash: "shell", shell: "shell", zsh: "shell" };

// Code -> HTML with spans for comments, strings, numbers and keywords (every piece escaped).
function highlight(code, lang) {
  const l = LANG_ALIASES[(lang || "").toLowerCase()];
  if (!l) return escapeHtml(code);
  const hashComments = l === "python" || l === "shell";
  const kw = new Set(KEYWORDS[l].split(" "));
  const re = hashComments
    ? /(#[^\n]*)|("""[\s\S]*?"""|'''[\s\S]*?'''|"(?:\\.|[^"\\\n])*"|'(?:\\.|[^'\\\n])*')|(\b\d+(?:\.\d+)?\b)|([A-Za-z_][A-Za-z0-9_]*)/g
    : /(\/\/[^\n]*|\/\*[\s\S]*?\*\/)|("(?:\\.|[^"\\\n])*"|'(?:\\.|[^'\\\n])*'|`(?:\\.|[^`\\])*`)|(\b\d+(?:\.\d+)?[fFuUlL]?\b)|([A-Za-z_][A-Za-z0-9_]*)/g;
  let out = "", last = 0, m;
  while ((m = re.exec(code)) !== null) {
    out += escapeHtml(code.slice(last, m.index));
    const t = escapeHtml(m[0]);
    if (m[1]) out += `<span class="hl-comment">${t}</span>`;
    else if (m[2]) out += `<span class="hl-string">${t}</span>`;
    else if (m[3]) out += `<span class="hl-number">${t}</span>`;
    else out += kw.has(m[4]) ? `<span class="hl-keyword">${t}</span>` : t;
    last = re.lastIndex;
  }
  return out + escapeHtml(code.slice(last));
}

// Inline markdown on ALREADY ESCAPED text: code spans, bold, italics, http(s) links.
function inline(s) {
  const codes = [];
  s = s.replace(/`([^`]+)`/g, (_, c) => { codes.push(c); return `\u0000${codes.length - 1}\u0000`; });
  s = s.replace(/\*\*([^*]+)\*\*/g, "<strong>$1</strong>").replace(/__([^_]+)__/g, "<strong>$1</strong>");
  s = s.replace(/(^|[^*])\*([^*\n]+)\*/g, "$1<em>$2</em>").replace(/(^|[^\w])_([^_\n]+)_(?!\w)/g, "$1<em>$2</em>");
  s = s.replace(/\[([^\]]+)\]\((https?:\/\/[^\s)]+)\)/g, '<a href="$2" target="_blank" rel="noopener noreferrer">$1</a>');
  return s.replace(/\u0000(\d+)\u0000/g, (_, i) => `<code>${codes[+i]}</code>`);
}

// Markdown -> HTML: fenced code blocks (language label + highlighting), headings, lists, block quotes, rules,
// paragraphs.  Everything the model wrote is escaped first: no raw HTML gets through.
function renderMarkdown(text) {
  const out = [];
  const parts = String(text).split(/^```/m);
  parts.forEach((p, i) => {
    if (i % 2 === 1) {  // fenced block: "lang\n body" (an unterminated fence while streaming is still code)
      const nl = p.indexOf("\n");
      const lang = nl >= 0 ? p.slice(0, nl).trim() : "";
      const body = (nl >= 0 ? p.slice(nl + 1) : "").replace(/\n$/, "");
      out.push(`<pre><div class="lang">${escapeHtml(lang || "code")}</div><code class="language-${escapeHtml(lang || "plain")}">` +
               `${highlight(body, lang)}</code></pre>`);
      return;
    }
    const lines = escapeHtml(p.replace(/^\n/, "")).split("\n");
    let list = null, para = [];
    const flushPara = () => { if (para.length) { out.push(`<p>${para.map(inline).join("<br>")}</p>`); para = []; } };
    const flushList = () => { if (list) { out.push(`<${list.tag}>${list.items.map((x) => `<li>${inline(x)}</li>`).join("")}</${list.tag}>`); list = null; } };
    for (const line of lines) {
      let m;
      if (!line.trim()) { flushPara(); flushList(); continue; }
      if ((m = line.match(/^(#{1,6})\s+(.*)$/))) { flushPara(); flushList(); out.push(`<h${m[1].length}>${inline(m[2])}</h${m[1].length}>`); continue; }
      if (/^(-{3,}|\*{3,})\s*$/.test(line)) { flushPara(); flushList(); out.push("<hr>"); continue; }
      if ((m = line.match(/^&gt;\s?(.*)$/))) { flushPara(); flushList(); out.push(`<blockquote>${inline(m[1])}</blockquote>`); continue; }
      if ((m = line.match(/^\s*([-*+]|\d+[.)])\s+(.*)$/))) {
        flushPara();
        const tag = /\d/.test(m[1]) ? "ol" : "ul";
        if (!list || list.tag !== tag) { flushList(); list = { tag, items: [] }; }
        list.items.push(m[2]);
        continue;
      }
      flushList();
      para.push(line);
    }
    flushPara(); flushList();
  });
  return out.join("");
}

// Conversation messages -> API messages.  A message carrying an attached image is sent as the reference UI
// sends it: [{type: image_url, image_url: {url: data URL}}, {type: text, text}] (the server keeps the last one).
function apiMessages(messages) {
  return messages.map((m) => (m.image
    ? { role: m.role, content: [{ type: "image_url", image_url: { url: m.image } }, { type: "text", text: m.content }] }
    : { role: m.role, content: m.content }));
}

function requestBody(model, messages, temperature, maxTokens) {
  return { model, stream: true, messages: apiMessages(messages), temperature, max_tokens: maxTokens };
}

// Resume decision for a failed send, called once per download-progress poll.  `w` = {failed, sawDownload,
// tries}: `failed` is set by the failed send; the pending message is re-sent only once a download was seen in
// progress AFTER that failure and every download has since completed (an empty progress map before any download
// was seen is not "complete"), and at most `maxTries` times per message.  Returns true to resume now.
function downloadComplete(d) {
  return d.status === "complete" || Boolean(d.total_bytes && d.downloaded_bytes >= d.total_bytes);
}

function resumeAfterDownload(w, entries, maxTries = 3) {
  if (!w.failed) return false;
  const active = entries.filter(([, d]) => !downloadComplete(d)).length;
  if (active > 0) { w.sawDownload = true; return false; }
  if (!w.sawDownload || w.tries >= maxTries) return false;
  w.failed = false; w.sawDownload = false; w.tries += 1;
  return true;
}

if (typeof module !== "undefined" && module.exports) {
  module.exports = { escapeHtml, highlight, renderMarkdown, apiMessages, requestBody, resumeAfterDownload };
}

// ------------------------------------------------------------------ the page
if (typeof window !== "undefined") {
const $ = (id) => document.getElementById(id);
const state = {
  histories: JSON.parse(localStorage.getItem("xot.histories") || "[]"),
  current: null,           // {id, title, model, messages: [{role, content, image?}]}
  models: {},              // id -> {name, downloaded, download_percentage, ...}
  model: localStorage.getItem("xot.model") || null,
  abort: null,
  image: null,             // data URL of the attachment for the next message
  lastError: null,         // the last send failed (e.g. the model was still downloading): resume when ready
  wait: { failed: false, sawDownload: false, tries: 0 },  // resumeAfterDownload's state for the pending message
};

function save() {
  // images make histories large: when localStorage is full, older conversations lose their image data first
  for (let drop = 0; drop <= state.histories.length; drop++) {
    try {
      const hs = state.histories.slice(0, 100).map((h, i) => (i < state.histories.length - drop ? h
        : { ...h, messages: h.messages.map(({ image, ...m }) => (image ? { ...m, content: m.content + " [image]" } : m)) }));
      localStorage.setItem("xot.histories", JSON.stringify(hs));
      break;
    } catch (e) { /* quota: retry with fewer images */ }
  }
  if (state.model) localStorage.setItem("xot.model", state.model);
}

function drawMessages() {
  const box = $("messages");
  box.innerHTML = "";
  const msgs = state.current ? state.current.messages : [];
  for (const m of msgs) {
    const d = document.createElement("div");
    d.className = `msg ${m.role}`;
    if (m.image) {
      const img = document.createElement("img");
      img.src = m.image;
      img.className = "attached";
      d.appendChild(img);
    }
    const body = document.createElement("div");
    body.innerHTML = m.role === "assistant" ? renderMarkdown(m.content) : escapeHtml(m.content);
    d.appendChild(body);
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

// ------------------------------------------------------------------ image attachment
function setImage(url) {
  state.image = url;
  const p = $("image-preview");
  p.hidden = !url;
  $("image-thumb").src = url || "";
}

function attachImage(ev) {
  const f = ev.target.files && ev.target.files[0];
  ev.target.value = "";
  if (!f) return;
  if (!f.type.startsWith("image/")) { $("stats").textContent = "not an image"; return; }
  const r = new FileReader();
  r.onload = (e) => setImage(e.target.result);
  r.readAsDataURL(f);
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
// The pending message: {conv, index} of the user message whose answer has not completed.  Kept across reloads
// and failed sends (the reference keeps it while a model downloads and re-sends it afterwards).
function setPending(p) {
  if (p) localStorage.setItem("xot.pending", JSON.stringify(p));
  else localStorage.removeItem("xot.pending");
}

function getPending() {
  try { return JSON.parse(localStorage.getItem("xot.pending") || "null"); } catch (e) { return null; }
}

async function send(text) {
  if ((!text.trim() && !state.image) || state.abort) return;
  if (!state.current) {
    state.current = { id: crypto.randomUUID ? crypto.randomUUID() : String(Date.now()),
                      title: (text || "image").slice(0, 40), model: state.model, messages: [] };
    state.histories.unshift(state.current);
  }
  const conv = state.current;
  const msg = { role: "user", content: text };
  if (state.image) { msg.image = state.image; setImage(null); }
  conv.messages.push(msg);
  setPending({ conv: conv.id, index: conv.messages.length - 1 });
  save();
  await generate(conv);
}

async function generate(conv) {
  const reply = { role: "assistant", content: "" };
  conv.messages.push(reply);
  drawHistory(); drawMessages();
  const ctrl = new AbortController();
  state.abort = ctrl;
  $("send").hidden = true; $("stop").hidden = false;
  const t0 = performance.now();
  let tFirst = null, nTok = 0, ok = false;
  const body = requestBody(state.model, conv.messages.slice(0, -1), parseFloat($("temperature").value),
                           parseInt($("max-tokens").value, 10));
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
    ok = true;
  } catch (e) {
    if (e.name === "AbortError") ok = true;  // stopped by the user: nothing to resume
    else {
      reply.content += `\n[error: ${e.message}]`; state.lastError = e.message;
      state.wait.failed = true; state.wait.sawDownload = false;
    }
  } finally {
    state.abort = null;
    if (ok) { setPending(null); state.lastError = null; state.wait = { failed: false, sawDownload: false, tries: 0 }; }
    $("send").hidden = false; $("stop").hidden = true;
    save(); drawMessages();
  }
}

// Re-send the pending message (after a reload, or once the downloads a failed send waited for are complete):
// the unanswered user message stays, the incomplete answer after it is replaced.
async function resumePending() {
  const p = getPending();
  if (!p || state.abort) return;
  const conv = state.histories.find((h) => h.id === p.conv);
  if (!conv || !conv.messages[p.index] || conv.messages[p.index].role !== "user") { setPending(null); return; }
  conv.messages.length = p.index + 1;
  state.current = conv;
  $("stats").textContent = "resuming the pending message…";
  await generate(conv);
}

// ------------------------------------------------------------------ ring / downloads panels
async function pollTopology() {
  try {
    const t = await (await fetch("/v1/topology")).json();
    const box = $("topology");
    box.innerHTML = "";
    const nodes = Object.entries(t.nodes || {});
    const layers = {};
    for (const p of t.partitions || []) layers[p.node_id] = `layers ${p.start_layer}-${p.end_layer}`;
    let tf = 0;
    for (const [id, c] of nodes) {
      tf += (c.flops && c.flops.fp16) || 0;
      const d = document.createElement("div");
      d.className = "peer" + (id === t.active_node_id ? " active" : "");
      d.textContent = `${id.slice(0, 20)} · ${c.chip} · ${(c.memory / 1024).toFixed(0)} GB` + (layers[id] ? ` · ${layers[id]}` : "");
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
    const entries = Object.entries(p);
    for (const [node, d] of entries) {
      const pct = d.total_bytes ? (100 * d.downloaded_bytes) / d.total_bytes : 0;
      const row = document.createElement("div");
      row.innerHTML = `<div class="muted">${escapeHtml(node.slice(0, 12))} ${escapeHtml(String(d.repo_id || ""))} ` +
        `${pct.toFixed(1)}%</div><div class="bar"><div style="width:${pct}%"></div></div>`;
      box.appendChild(row);
    }
    if (getPending() && resumeAfterDownload(state.wait, entries)) { state.lastError = null; resumePending(); }
  } catch (e) { /* ignore */ }
}

// ------------------------------------------------------------------ wiring
window.addEventListener("DOMContentLoaded", () => {
  $("new-chat").onclick = newChat;
  $("model-select").onchange = (e) => { state.model = e.target.value; save(); drawModels(); };
  $("download-model").onclick = downloadModel;
  $("delete-model").onclick = deleteModel;
  $("stop").onclick = () => state.abort && state.abort.abort();
  $("attach").onclick = () => $("image-input").click();
  $("image-input").onchange = attachImage;
  $("image-clear").onclick = () => setImage(null);
  $("composer").onsubmit = (e) => { e.preventDefault(); const v = $("prompt").value; $("prompt").value = ""; send(v); };
  $("prompt").addEventListener("keydown", (e) => {
    if (e.key === "Enter" && !e.shiftKey) { e.preventDefault(); $("composer").requestSubmit(); }
  });
  drawHistory(); drawMessages();
  loadModels().then(() => { if (getPending()) resumePending(); });
  pollTopology(); setInterval(pollTopology, 5000);
  pollDownloads(); setInterval(pollDownloads, 1000);
});
}
