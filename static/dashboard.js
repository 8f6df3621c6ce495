// Training dashboard (reference static/dashboard.js): polls /progress and /stats for a model and
// renders cost curves, weight-update ratios and per-layer activation / gradient / weight-gradient
// statistics. Data contract identical to the reference service; charts drawn by static/plot.js.

const qs = name => new URLSearchParams(window.location.search).get(name);

function setQueryParam(name, value) {
    const url = new URL(window.location);
    url.searchParams.set(name, value);
    window.history.replaceState({}, '', url);
}

function heading(container, tag, text) {
    const el = document.createElement(tag);
    el.textContent = text;
    container.appendChild(el);
}

function lineChart(container, lists, labelOf, title, fmtX, fmtY) {
    const datasets = [];
    lists.forEach((data, i) => { if (data) datasets.push({ label: labelOf(i), data }); });
    PzPlot.plot({ container, datasets, title, formatX: fmtX, formatY: fmtY });
}

function histogramChart(container, hists, labelOf, title, fmtX, fmtY) {
    const datasets = [];
    hists.forEach((h, i) => {
        if (h) datasets.push({ label: labelOf(i), data: h.x.map((x, k) => ({ x, y: h.y[k] })) });
    });
    PzPlot.plot({ container, datasets, title, stacked: true, formatX: fmtX, formatY: fmtY });
}

async function fetchJson(path, modelId) {
    const res = await fetch(`${path}?model_id=${encodeURIComponent(modelId)}`);
    if (!res.ok) throw new Error(path);
    return res.json();
}

async function refresh() {
    const modelId = document.getElementById('model-id').value.trim();
    if (!modelId) { alert('Please enter a model ID.'); return; }
    setQueryParam('model_id', modelId);
    const filterText = document.getElementById('layer-filter').value.trim().toLowerCase();
    setQueryParam('layer', filterText);

    let progress, stats;
    try { progress = await fetchJson('/progress/', modelId); }
    catch (e) { alert('Failed to fetch progress. Check model ID.'); return; }
    if (!progress) return;
    try { stats = await fetchJson('/stats/', modelId); }
    catch (e) { alert('Failed to fetch stats. Check model ID.'); return; }

    const box = document.getElementById('data-container');
    box.innerHTML = '';
    const f0 = x => x.toFixed(0), f4 = y => y.toFixed(4);

    heading(box, 'h2', `Cost progress for model ${modelId}`);
    heading(box, 'h3', `Average Cost: ${progress.average_cost}  —  status: ${progress.status}`);
    lineChart(box, [progress.progress.map(p => ({ x: p.epoch, y: Math.log10(p.cost) }))],
              () => 'Cost progress', 'Cost Progression (Log Scale)', f0, f4);
    lineChart(box, [progress.average_cost_history.map((c, i) => ({ x: i, y: Math.log10(c) }))],
              () => 'Overall Average Cost', 'Average Cost Overall (Log Scale)', f0, f4);

    // layer filter: comma separated layer indices or algo substrings
    const filters = filterText.split(',').map(s => s.trim()).filter(s => s.length);
    const layerOk = (layer, i) => !filters.length || filters.some(f => f == i || (layer && layer.algo.includes(f)));
    const indexOk = i => layerOk(stats ? stats.layers[i] : null, i);

    heading(box, 'h2', `Weight updates for model ${modelId}`);
    const ratioLists = [];
    progress.progress.forEach(p => (p.weight_upd_ratio || []).forEach((r, i) => {
        if (r && indexOk(i)) (ratioLists[i] ??= []).push({ x: p.epoch, y: Math.log10(r) });
    }));
    lineChart(box, ratioLists, i => `Weights ${i}`, 'Weight Update Std Ratio (Log Scale)', f0, f4);

    if (!stats) return;
    const layers = stats.layers.map((l, i) => ({ l, i })).filter(({ l, i }) => layerOk(l, i));

    heading(box, 'h2', `Activations for model ${modelId}`);
    layers.forEach(({ l, i }) => {
        const a = l.activation;
        heading(box, 'h3', `Layer ${i} (${l.algo}): mean ${a.mean.toFixed(2)} std ${a.std.toFixed(2)} ` +
                           `saturated: ${(a.saturated * 100).toFixed(1)}%`);
    });
    histogramChart(box, layers.map(({ l }) => l.activation.histogram), k => `Layer ${layers[k].i} (${layers[k].l.algo})`,
                   'Activation Distribution', null, f4);

    heading(box, 'h2', `Gradients for model ${modelId}`);
    layers.forEach(({ l, i }) => {
        if (l.gradient) heading(box, 'h3', `Layer ${i} (${l.algo}): mean ${l.gradient.mean.toExponential(6)} ` +
                                           `std ${l.gradient.std.toExponential(6)}`);
    });
    histogramChart(box, layers.map(({ l }) => l.gradient && l.gradient.histogram),
                   k => `Layer ${layers[k].i} (${layers[k].l.algo})`, 'Gradient Distribution', x => x.toFixed(6), f4);

    heading(box, 'h2', `Weights for model ${modelId}`);
    const weights = stats.weights.map((w, i) => (indexOk(i) ? w : null));
    weights.forEach((w, i) => {
        if (!w) return;
        const ratio = (w.gradient.std / w.data.std).toExponential(6);
        heading(box, 'h3', `Weights ${i} - ${w.shape}: mean ${w.gradient.mean.toExponential(6)} ` +
                           `std ${w.gradient.std.toExponential(6)}  grad:data ratio ${ratio}`);
    });
    histogramChart(box, weights.map(w => w && w.gradient.histogram), i => `Weights ${i} - ${weights[i].shape}`,
                   'Weight Gradient Distribution', x => x.toFixed(3), f4);
}

let timer = null;
window.onload = () => {
    const id = qs('model_id');
    if (id) document.getElementById('model-id').value = id;
    const layer = qs('layer');
    if (layer) document.getElementById('layer-filter').value = layer;
    document.getElementById('auto-refresh').addEventListener('change', ev => {
        if (timer) { clearInterval(timer); timer = null; }
        if (ev.target.checked) timer = setInterval(refresh, 5000);
    });
};
