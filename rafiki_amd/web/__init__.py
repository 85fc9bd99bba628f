"""Admin web dashboard: one static page served by the admin at ``/ui`` (no Node build step).

Reference: web/ (React + Material-UI + echarts SPA, ~1.1k LoC TS; server web/app.js).  Same pages
and routes — login, train jobs of the user, a train job with its trials, a trial with its
messages and metric plots built from the ModelLogger PLOT/METRICS lines exactly as
web/src/pages/train/TrialDetailPage.tsx:205-262 does (x = plot.x_axis or time) — plus the user's
inference jobs.  Plots are rendered as inline SVG.  The page talks to the same REST API as the
Python client (Bearer JWT from POST /tokens, kept in localStorage).
"""

INDEX_HTML = r"""<!doctype html>
<html lang="en"><head><meta charset="utf-8"><title>Rafiki (MI355X) admin</title>
<meta name="viewport" content="width=device-width, initial-scale=1">
<style>
body{font-family:system-ui,-apple-system,Segoe UI,Roboto,sans-serif;margin:0;background:#f4f5f7;color:#222}
header{background:#1f2937;color:#fff;padding:10px 20px;display:flex;justify-content:space-between;align-items:center}
header a{color:#cbd5e1;margin-left:16px;text-decoration:none}
main{padding:20px;max-width:1200px;margin:auto}
table{border-collapse:collapse;width:100%;background:#fff;margin-bottom:20px}
th,td{border-bottom:1px solid #e5e7eb;padding:6px 10px;text-align:left;font-size:14px;vertical-align:top}
th{background:#f9fafb}
.card{background:#fff;padding:16px;margin-bottom:16px;border-radius:6px;box-shadow:0 1px 2px rgba(0,0,0,.08)}
input{padding:6px;margin:4px 0;width:260px} button{padding:6px 14px;cursor:pointer}
.err{color:#b91c1c} .muted{color:#6b7280;font-size:13px} code{font-size:12px}
.plots{display:flex;flex-wrap:wrap;gap:16px} .plot{background:#fff;padding:8px;border-radius:6px}
.st-RUNNING{color:#047857}.st-ERRORED{color:#b91c1c}.st-STOPPED,.st-COMPLETED{color:#374151}
</style></head><body>
<header><b>Rafiki admin</b><nav id="nav"></nav></header>
<main id="app"></main>
<script>
const API = window.location.origin;
const S = {token: localStorage.getItem('rk_token'), user: JSON.parse(localStorage.getItem('rk_user')||'null')};
const $ = (h) => { document.getElementById('app').innerHTML = h; };
const esc = (s) => String(s===null||s===undefined?'':s).replace(/[&<>"']/g, c => ({'&':'&amp;','<':'&lt;','>':'&gt;','"':'&quot;',"'":'&#39;'}[c]));
async function api(method, path, body) {
  const opt = {method, headers: {'Content-Type': 'application/json'}};
  if (S.token) opt.headers['Authorization'] = 'Bearer ' + S.token;
  if (body) opt.body = JSON.stringify(body);
  const r = await fetch(API + path, opt);
  const t = await r.text();
  let d; try { d = JSON.parse(t); } catch (e) { d = t; }
  if (!r.ok) throw new Error((d && d.error) || t || r.status);
  return d;
}
function nav() {
  document.getElementById('nav').innerHTML = S.token
    ? `<span class="muted">${esc(S.user && S.user.user_type)}</span><a href="#/train-jobs">Train jobs</a><a href="#/inference-jobs">Inference jobs</a><a href="#/logout">Logout</a>`
    : '';
}
function fmtTime(t) { return t ? esc(String(t).replace('T', ' ').slice(0, 19)) : '-'; }
function statusCell(s) { return `<span class="st-${esc(s)}">${esc(s)}</span>`; }

async function loginPage(msg) {
  $(`<div class="card"><h3>Sign in</h3><div class="err">${esc(msg||'')}</div>
     <input id="em" placeholder="email" value="superadmin@rafiki"><br><input id="pw" type="password" placeholder="password"><br>
     <button id="go">Login</button></div>`);
  document.getElementById('go').onclick = async () => {
    try {
      const d = await api('POST', '/tokens', {email: document.getElementById('em').value, password: document.getElementById('pw').value});
      S.token = d.token; S.user = d; localStorage.setItem('rk_token', d.token); localStorage.setItem('rk_user', JSON.stringify(d));
      location.hash = '#/train-jobs';
    } catch (e) { loginPage(e.message); }
  };
}
async function trainJobsPage() {
  const jobs = await api('GET', '/train_jobs?user_id=' + encodeURIComponent(S.user.user_id));
  const rows = jobs.map(j => `<tr><td><a href="#/train-jobs/${encodeURIComponent(j.app)}/${j.app_version}">${esc(j.app)}</a></td><td>${j.app_version}</td>
     <td>${esc(j.task)}</td><td>${statusCell(j.status)}</td><td><code>${esc(JSON.stringify(j.budget))}</code></td><td>${fmtTime(j.datetime_started)}</td><td>${fmtTime(j.datetime_stopped)}</td></tr>`).join('');
  $(`<h2>Train jobs</h2><table><tr><th>App</th><th>Version</th><th>Task</th><th>Status</th><th>Budget</th><th>Started</th><th>Stopped</th></tr>${rows || '<tr><td colspan=7 class="muted">none</td></tr>'}</table>`);
}
async function trainJobPage(app, ver) {
  const [tj, trials] = await Promise.all([api('GET', `/train_jobs/${encodeURIComponent(app)}/${ver}`),
                                          api('GET', `/train_jobs/${encodeURIComponent(app)}/${ver}/trials`)]);
  const workers = (tj.workers||[]).map(w => `<tr><td>${esc(w.model_name)}</td><td>${statusCell(w.status)}</td><td>${fmtTime(w.datetime_started)}</td><td>${fmtTime(w.datetime_stopped)}</td></tr>`).join('');
  const rows = trials.map((t, i) => `<tr><td>${trials.length - i}</td><td><a href="#/trial/${esc(t.id)}">${esc(t.id.slice(0, 8))}</a></td><td>${esc(t.model_name)}</td>
     <td>${statusCell(t.status)}</td><td>${t.score===null||t.score===undefined?'-':Number(t.score).toFixed(4)}</td><td><code>${esc(JSON.stringify(t.knobs))}</code></td><td>${fmtTime(t.datetime_started)}</td><td>${fmtTime(t.datetime_stopped)}</td></tr>`).join('');
  $(`<h2>${esc(app)} v${esc(ver)}</h2><div class="card">Status ${statusCell(tj.status)} &middot; task ${esc(tj.task)} &middot; budget <code>${esc(JSON.stringify(tj.budget))}</code>
     <div class="muted">train ${esc(tj.train_dataset_uri)} &middot; test ${esc(tj.test_dataset_uri)}</div></div>
     <h3>Workers</h3><table><tr><th>Model</th><th>Status</th><th>Started</th><th>Stopped</th></tr>${workers}</table>
     <h3>Trials</h3><table><tr><th>#</th><th>ID</th><th>Model</th><th>Status</th><th>Score</th><th>Knobs</th><th>Started</th><th>Stopped</th></tr>${rows}</table>`);
}
function plotSvg(plot, metrics) {
  const xAxis = plot.x_axis || 'time';
  const series = plot.metrics.map(() => []);
  for (const m of metrics) {
    if (!(xAxis in m)) continue;
    const x = xAxis === 'time' ? Date.parse(m.time) : Number(m[xAxis]);
    plot.metrics.forEach((k, i) => { if (k in m && m[k] !== null) series[i].push([x, Number(m[k])]); });
  }
  const pts = series.flat();
  if (!pts.length) return `<div class="plot"><b>${esc(plot.title)}</b><div class="muted">no data</div></div>`;
  const W = 520, H = 260, P = 40;
  let [x0, x1] = [Math.min(...pts.map(p => p[0])), Math.max(...pts.map(p => p[0]))];
  let [y0, y1] = [Math.min(...pts.map(p => p[1])), Math.max(...pts.map(p => p[1]))];
  if (x1 === x0) x1 = x0 + 1; if (y1 === y0) { y1 = y0 + 1; y0 = y0 - 1; }
  const sx = x => P + (x - x0) / (x1 - x0) * (W - 2 * P), sy = y => H - P - (y - y0) / (y1 - y0) * (H - 2 * P);
  const colors = ['#2563eb', '#dc2626', '#059669', '#d97706', '#7c3aed'];
  const lines = series.map((s, i) => `<polyline fill="none" stroke="${colors[i % 5]}" stroke-width="2" points="${s.map(p => sx(p[0]).toFixed(1) + ',' + sy(p[1]).toFixed(1)).join(' ')}"/>` +
      s.map(p => `<circle cx="${sx(p[0]).toFixed(1)}" cy="${sy(p[1]).toFixed(1)}" r="2.5" fill="${colors[i % 5]}"><title>${esc(plot.metrics[i])}=${p[1]}</title></circle>`).join('')).join('');
  const legend = plot.metrics.map((k, i) => `<tspan fill="${colors[i % 5]}">&#9632; ${esc(k)} </tspan>`).join('');
  return `<div class="plot"><svg width="${W}" height="${H}" xmlns="http://www.w3.org/2000/svg">
    <text x="${P}" y="16" font-weight="bold">${esc(plot.title)}</text><text x="${W - P}" y="16" text-anchor="end" font-size="12">${legend}</text>
    <line x1="${P}" y1="${H - P}" x2="${W - P}" y2="${H - P}" stroke="#9ca3af"/><line x1="${P}" y1="${P}" x2="${P}" y2="${H - P}" stroke="#9ca3af"/>
    <text x="${P}" y="${H - P + 16}" font-size="11">${xAxis === 'time' ? '' : esc(x0.toPrecision(4))}</text>
    <text x="${W - P}" y="${H - P + 16}" font-size="11" text-anchor="end">${esc(xAxis)} ${xAxis === 'time' ? '' : esc(x1.toPrecision(4))}</text>
    <text x="4" y="${H - P}" font-size="11">${esc(y0.toPrecision(4))}</text><text x="4" y="${P + 4}" font-size="11">${esc(y1.toPrecision(4))}</text>
    ${lines}</svg></div>`;
}
async function trialPage(id) {
  const [t, logs] = await Promise.all([api('GET', '/trials/' + encodeURIComponent(id)), api('GET', '/trials/' + encodeURIComponent(id) + '/logs')]);
  const msgs = (logs.messages || []).map(m => `<tr><td>${fmtTime(m.time)}</td><td>${esc(m.message)}</td></tr>`).join('');
  const plots = (logs.plots || []).map(p => plotSvg(p, logs.metrics || [])).join('');
  $(`<h2>Trial ${esc(id)}</h2><div class="card">Model ${esc(t.model_name)} &middot; ${statusCell(t.status)} &middot; score ${t.score===null||t.score===undefined?'-':esc(t.score)}
     <div><code>${esc(JSON.stringify(t.knobs))}</code></div><div class="muted">${fmtTime(t.datetime_started)} &rarr; ${fmtTime(t.datetime_stopped)}</div></div>
     <h3>Plots</h3><div class="plots">${plots || '<span class="muted">no plots</span>'}</div>
     <h3>Messages</h3><table><tr><th>Time</th><th>Message</th></tr>${msgs}</table>`);
}
async function inferenceJobsPage() {
  const jobs = await api('GET', '/inference_jobs?user_id=' + encodeURIComponent(S.user.user_id));
  const rows = jobs.map(j => `<tr><td>${esc(j.app)}</td><td>${j.app_version}</td><td>${statusCell(j.status)}</td><td>${esc(j.predictor_host || '-')}</td><td>${fmtTime(j.datetime_started)}</td><td>${fmtTime(j.datetime_stopped)}</td></tr>`).join('');
  $(`<h2>Inference jobs</h2><table><tr><th>App</th><th>Version</th><th>Status</th><th>Predictor</th><th>Started</th><th>Stopped</th></tr>${rows || '<tr><td colspan=6 class="muted">none</td></tr>'}</table>`);
}
async function route() {
  nav();
  const h = location.hash.replace(/^#/, '') || '/train-jobs';
  if (h === '/logout') { S.token = null; S.user = null; localStorage.clear(); location.hash = '#/login'; return; }
  if (!S.token || h === '/login') return loginPage();
  try {
    let m;
    if ((m = h.match(/^\/train-jobs\/([^/]+)\/([^/]+)$/))) return await trainJobPage(decodeURIComponent(m[1]), m[2]);
    if ((m = h.match(/^\/trial\/([^/]+)$/))) return await trialPage(decodeURIComponent(m[1]));
    if (h === '/inference-jobs') return await inferenceJobsPage();
    return await trainJobsPage();
  } catch (e) {
    if (/token|auth|401|403/i.test(e.message)) return loginPage(e.message);
    $(`<div class="err">${esc(e.message)}</div>`);
  }
}
window.addEventListener('hashchange', route);
route();
</script></body></html>
"""
