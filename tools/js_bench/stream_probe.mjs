// detectAsync with keypoint objects, 3 in flight, each result awaited in order: per-job latency and JS work.
import fs from 'fs';
import { performance } from 'perf_hooks';
import * as sift from '../../sift-scale-space-extrema-detection_amd/js/sift.mjs';
const [, , inPath, Ws, Hs] = process.argv;
const W = +Ws, H = +Hs;
const raw = fs.readFileSync(inPath);
const image = { width: W, height: H, data: new Float32Array(raw.buffer, raw.byteOffset, W * H) };
const opts = { number_of_octaves: 4, scales_per_octave: 5 };
(async () => {
  for (let i = 0; i < 3; i++) await sift.detectAsync(image, opts);
  for (const depth of [3, 1]) {
    global.gc && global.gc();
    const q = [], lat = [];
    const t0 = performance.now();
    for (let i = 0; i < 30; i++) {
      const ts = performance.now();
      q.push(sift.detectAsync(image, opts).then((r) => { lat.push(performance.now() - ts); return r; }));
      if (q.length === depth) await q.shift();
    }
    while (q.length) await q.shift();
    const ms = (performance.now() - t0) / 30;
    lat.sort((a, b) => a - b);
    console.log(`depth ${depth}: ${ms.toFixed(2)} ms/image, job latency median ${lat[15].toFixed(2)} max ${lat[29].toFixed(2)}`);
  }
  global.gc && global.gc();
  let t0 = performance.now();
  for (let i = 0; i < 30; i++) sift.detect(image, opts);
  console.log(`sync: ${((performance.now() - t0) / 30).toFixed(2)} ms/image`);
})();
