// Minimal dependency-free canvas plotting for the training dashboard.
//
// Replaces the reference's vendored Chart.js (static/chart-4.4.1.umd.min.js, 200 KB) with the
// two chart forms the dashboard actually uses: multi-series line charts on linear axes and
// stacked, filled histogram curves. Data points are {x, y} objects (Chart.js `parsing: false`
// style), the Y range gets 5 % padding (0.1 for flat lines), hovering shows the nearest point.
(function (global) {
    const PALETTE = ['#3366cc', '#dc3912', '#ff9900', '#109618', '#990099', '#0099c6', '#dd4477',
                     '#66aa00', '#b82e2e', '#316395', '#994499', '#22aa99', '#aaaa11', '#6633cc'];

    function niceTicks(lo, hi, count) {
        if (!(hi > lo)) return [lo];
        const raw = (hi - lo) / Math.max(1, count);
        const mag = Math.pow(10, Math.floor(Math.log10(raw)));
        const step = [1, 2, 2.5, 5, 10].map(m => m * mag).find(s => s >= raw) || raw;
        const ticks = [];
        for (let v = Math.ceil(lo / step) * step; v <= hi + step * 1e-9; v += step) ticks.push(v);
        return ticks;
    }

    function plot({ container, datasets, title, stacked = false, formatX = null, formatY = null }) {
        datasets = datasets.filter(d => d && d.data && d.data.length);
        const wrap = document.createElement('div');
        wrap.className = 'plot';
        const canvas = document.createElement('canvas');
        const W = 800, H = 400;
        const dpr = global.devicePixelRatio || 1;
        canvas.width = W * dpr; canvas.height = H * dpr;
        canvas.style.width = W + 'px'; canvas.style.height = H + 'px';
        const tip = document.createElement('div');
        tip.className = 'tip';
        wrap.appendChild(canvas); wrap.appendChild(tip);
        container.appendChild(wrap);
        const ctx = canvas.getContext('2d');
        ctx.scale(dpr, dpr);

        // stacking by point index (as Chart.js stacks datasets)
        const series = datasets.map(d => d.data.map(p => ({ x: p.x, y: p.y, y0: 0 })));
        if (stacked) {
            for (let s = 1; s < series.length; s++)
                series[s].forEach((p, i) => {
                    const below = series[s - 1][i];
                    p.y0 = below ? below.y0 + below.y : 0;
                });
        }
        const xs = series.flatMap(s => s.map(p => p.x)).filter(Number.isFinite);
        const ys = series.flatMap(s => s.map(p => p.y + p.y0)).filter(Number.isFinite);
        if (stacked) ys.push(0);
        const pad = { l: 70, r: 20, t: title ? 40 : 15, b: 40 };
        ctx.font = '12px sans-serif';
        if (title) {
            ctx.font = 'bold 16px sans-serif';
            ctx.fillStyle = '#222';
            ctx.textAlign = 'center';
            ctx.fillText(title, W / 2, 24);
            ctx.font = '12px sans-serif';
        }
        if (!xs.length || !ys.length) {
            ctx.fillStyle = '#888'; ctx.textAlign = 'center';
            ctx.fillText('no data', W / 2, H / 2);
            return;
        }
        let minX = Math.min(...xs), maxX = Math.max(...xs);
        let minY = Math.min(...ys), maxY = Math.max(...ys);
        if (maxX === minX) { minX -= 0.5; maxX += 0.5; }
        const yPad = maxY === minY ? 0.1 : (maxY - minY) * 0.05;
        minY -= yPad; maxY += yPad;
        const px = x => pad.l + (x - minX) / (maxX - minX) * (W - pad.l - pad.r);
        const py = y => H - pad.b - (y - minY) / (maxY - minY) * (H - pad.t - pad.b);

        // axes + grid
        ctx.strokeStyle = '#e5e5e5'; ctx.fillStyle = '#555'; ctx.lineWidth = 1;
        ctx.textAlign = 'right';
        niceTicks(minY, maxY, 6).forEach(v => {
            ctx.beginPath(); ctx.moveTo(pad.l, py(v)); ctx.lineTo(W - pad.r, py(v)); ctx.stroke();
            ctx.fillText(formatY ? formatY(v) : String(+v.toPrecision(4)), pad.l - 6, py(v) + 4);
        });
        ctx.textAlign = 'center';
        niceTicks(minX, maxX, 10).forEach(v => {
            ctx.beginPath(); ctx.moveTo(px(v), pad.t); ctx.lineTo(px(v), H - pad.b); ctx.stroke();
            ctx.fillText(formatX ? formatX(v) : v.toFixed(2), px(v), H - pad.b + 16);
        });
        ctx.strokeStyle = '#888';
        ctx.strokeRect(pad.l, pad.t, W - pad.l - pad.r, H - pad.t - pad.b);

        // series
        series.forEach((pts, s) => {
            const color = PALETTE[s % PALETTE.length];
            const ok = pts.filter(p => Number.isFinite(p.x) && Number.isFinite(p.y));
            if (!ok.length) return;
            ctx.beginPath();
            ok.forEach((p, i) => (i ? ctx.lineTo : ctx.moveTo).call(ctx, px(p.x), py(p.y + p.y0)));
            if (stacked) {
                for (let i = ok.length - 1; i >= 0; i--) ctx.lineTo(px(ok[i].x), py(ok[i].y0));
                ctx.closePath();
                ctx.globalAlpha = 0.25; ctx.fillStyle = color; ctx.fill(); ctx.globalAlpha = 1;
                ctx.beginPath();
                ok.forEach((p, i) => (i ? ctx.lineTo : ctx.moveTo).call(ctx, px(p.x), py(p.y + p.y0)));
            }
            ctx.strokeStyle = color; ctx.lineWidth = 2; ctx.stroke();
        });

        // legend
        ctx.textAlign = 'left';
        let lx = pad.l + 8, ly = pad.t + 14;
        datasets.forEach((d, s) => {
            const label = d.label || `series ${s}`;
            const w = ctx.measureText(label).width + 26;
            if (lx + w > W - pad.r) { lx = pad.l + 8; ly += 16; }
            ctx.fillStyle = PALETTE[s % PALETTE.length]; ctx.fillRect(lx, ly - 9, 12, 10);
            ctx.fillStyle = '#222'; ctx.fillText(label, lx + 16, ly);
            lx += w;
        });

        // hover: nearest point
        canvas.addEventListener('mousemove', ev => {
            const r = canvas.getBoundingClientRect();
            const mx = ev.clientX - r.left, my = ev.clientY - r.top;
            let best = null;
            series.forEach((pts, s) => pts.forEach(p => {
                const d = Math.hypot(px(p.x) - mx, py(p.y + p.y0) - my);
                if (Number.isFinite(d) && (!best || d < best.d)) best = { d, s, p };
            }));
            if (!best || best.d > 30) { tip.style.display = 'none'; return; }
            const label = datasets[best.s].label || '';
            tip.textContent = `${label}: (${formatX ? formatX(best.p.x) : best.p.x}, ` +
                              `${formatY ? formatY(best.p.y) : best.p.y})`;
            tip.style.left = (mx + 12) + 'px'; tip.style.top = (my - 10) + 'px';
            tip.style.display = 'block';
        });
        canvas.addEventListener('mouseleave', () => { tip.style.display = 'none'; });
    }

    global.PzPlot = { plot };
})(window);
