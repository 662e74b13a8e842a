// Queued detectAsync per image at several pool sizes: node inflight_probe.mjs <img.f32> W H [format]
import fs from 'fs';
import { performance } from 'perf_hooks';
import * as sift from '../../sift-scale-space-extrema-detection_amd/js/sift.mjs';
const [, , inPath, Ws, Hs, fmt = 'typed'] = process.argv;
const W = +Ws, H = +Hs;
const raw = fs.readFileSync(inPath);
const image = { width: W, height: H, data: new Float32Array(raw.buffer, raw.byteOffset, W * H) };
const base = { number_of_octaves: 4, scales_per_octave: 5, format: fmt };
(async () => {
  for (const inflight of (process.env.POOLS || "3,4,3,4,3,4").split(",").map(Number)) {
    const o = { ...base, inflight };
    await Promise.all(Array.from({ length: inflight }, () => sift.detectAsync(image, o)));
    const t0 = performance.now();
    let rs = await Promise.all(Array.from({ length: 40 }, () => sift.detectAsync(image, o)));
    const ms = (performance.now() - t0) / 40;
    rs = null;
    if (global.gc) global.gc();
    console.log(`${W}x${H} ${fmt} inflight ${inflight}: ${ms.toFixed(3)} ms/image, ${(W * H / 1e3 / ms).toFixed(0)} Mpix/s`);
  }
})();
