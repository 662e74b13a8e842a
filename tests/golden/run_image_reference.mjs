// Golden-vector generator for the image products either side of the path
// (SURVEY.md §8f rows 2-3): imports the UNMODIFIED reference modules
// /root/reference/src/image-utils.js and src/matrix2d.js and runs
//   ImageUtils_convertImageDataToMatrix2D (gray + alpha, perceptual, as main.js:98-103)
//   ImageUtils_convertMatrix2DToImageData of the plain, Matrix2D_sigmoidNormalize(.., c)
//   and Matrix2D_sampledNormalize forms of a matrix (background.js:139, :303, :336)
// on inputs given as raw files.  Run only in the build container by
// make_image_golden.py (OffscreenCanvas is an inert stub, as in
// run_reference.mjs).
//
// usage: node --experimental-loader ./ref_loader.mjs run_image_reference.mjs \
//          <rgba.u8> <W> <H> <matrix.f32> <MW> <MH> <coef> <outdir>
import fs from 'fs';
import path from 'path';

const [, , rgbaPath, W_, H_, matPath, MW_, MH_, coef_, outDir] = process.argv;
const W = +W_, H = +H_, MW = +MW_, MH = +MH_, coef = +coef_;

globalThis.OffscreenCanvas = class {
  constructor(w, h) { this.w = w; this.h = h; }
  getContext() {
    return { createImageData: (w, h) => ({ width: w, height: h, data: new Uint8ClampedArray(w * h * 4) }) };
  }
};

import('/root/reference/src/image-utils.js').then(async (IU) => {
  const M = await import('/root/reference/src/matrix2d.js');
  const raw = fs.readFileSync(rgbaPath);
  const imageData = { width: W, height: H, data: new Uint8ClampedArray(raw.buffer, raw.byteOffset, W * H * 4) };
  const [gray, alpha] = IU.ImageUtils_convertImageDataToMatrix2D({
    imageData, convertToGrayscale: true, usePerceptualGrayscale: true,
  });
  const g64 = new Float64Array(W * H), a64 = new Float64Array(W * H);
  for (let y = 0; y < H; y++) for (let x = 0; x < W; x++) { g64[y * W + x] = gray[y][x]; a64[y * W + x] = alpha[y][x]; }
  fs.writeFileSync(path.join(outDir, 'gray.f64'), Buffer.from(g64.buffer));
  fs.writeFileSync(path.join(outDir, 'alpha.f64'), Buffer.from(a64.buffer));

  const mraw = fs.readFileSync(matPath);
  const f32 = new Float32Array(mraw.buffer, mraw.byteOffset, MW * MH);
  const mat = [];
  for (let y = 0; y < MH; y++) { const r = []; for (let x = 0; x < MW; x++) r.push(f32[y * MW + x]); mat.push(r); }
  const forms = {
    plain: mat,
    sigmoid: M.Matrix2D_sigmoidNormalize(mat, coef),
    sampled: M.Matrix2D_sampledNormalize(mat),
  };
  for (const [name, m] of Object.entries(forms)) {
    const img = IU.ImageUtils_convertMatrix2DToImageData(MW, MH, { grayChannelMatrix: m });
    fs.writeFileSync(path.join(outDir, name + '.u8'), Buffer.from(img.data.buffer));
  }
});
