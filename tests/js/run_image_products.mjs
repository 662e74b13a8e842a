// Drives the JS image products (SURVEY.md §8f rows 2-3) for
// tests/test_js.py: RGBA ImageData -> gray (convertImageDataToMatrix2D),
// preview ImageData of a caller-supplied plane (planeImageData in all three
// display modes), RGBA input to the stage chain and the one-call path, and
// the worker protocol's preview messages.
// usage: node run_image_products.mjs <rgba.u8> <W> <H> <matrix.f32> <out.json>
import fs from 'fs';
import * as sift from '../../sift-scale-space-extrema-detection_amd/js/sift.mjs';

const [, , rgbaPath, W_, H_, matPath, outPath] = process.argv;
const W = +W_, H = +H_;
const raw = fs.readFileSync(rgbaPath);
const imageData = { width: W, height: H, data: new Uint8ClampedArray(raw.buffer, raw.byteOffset, W * H * 4) };
const out = {};

// image-utils.js:27-152 (as main.js:98-103 calls it)
const [gray, alpha] = sift.convertImageDataToMatrix2D({ imageData, convertToGrayscale: true,
  usePerceptualGrayscale: true, matrix2d: false });
out.gray = Array.from(gray.data);
out.alpha = Array.from(alpha.data);
const g2 = sift.convertImageDataToMatrix2D({ imageData, convertToGrayscale: true, discardAlphaChannel: true });
out.grayRows = g2.length;
out.grayRow0 = g2[0];

// previews of a caller-supplied plane: a foreign DoG pyramid (1 octave, S = 1)
const mraw = fs.readFileSync(matPath);
const mat = new Float32Array(mraw.buffer, mraw.byteOffset, 4 * W * H);
const plane = (k) => ({ blurLevel: 1, image: { width: 2 * W, height: 2 * H, data: Float32Array.from(mat, v => v * k) } });
const dog = [[plane(1), plane(0.5), plane(0.25)]];
sift.findCandidateKeypoints(dog, null, 1);
out.images = {};
for (const mode of ['plain', 'sigmoid', 'sampled']) {
  const img = sift.planeImageData(dog, 0, 0, { mode, coefficient: 5 });
  out.images[mode] = { width: img.width, height: img.height, clamped: img.data instanceof Uint8ClampedArray,
    data: Array.from(img.data) };
}

// RGBA straight into the path
const params = { number_of_octaves: 3, scales_per_octave: 3 };
out.detectRgba = sift.detect(imageData, params).map(k => [k.absoluteX, k.absoluteY, k.absoluteSigma]);
out.detectGray = sift.detect(gray, params).map(k => [k.absoluteX, k.absoluteY, k.absoluteSigma]);
const ss = sift.computeGaussianScaleSpace({ input_image: imageData, number_of_octaves: 3, scales_per_octave: 3 });
out.ssSample = Array.from(ss[1][2].image.data.subarray(0, 32));
const ssg = sift.computeGaussianScaleSpace({ input_image: gray, number_of_octaves: 3, scales_per_octave: 3 });
out.ssSampleGray = Array.from(ssg[1][2].image.data.subarray(0, 32));

// worker protocol with previews (background.js message order)
const posted = [];
const onmessage = sift.createWorkerHandler(m => posted.push(m), { matrix2d: true, previews: true, chunks: false });
onmessage({ data: { type: sift.WorkerMessageTypes.COMPUTE_GAUSSIAN_SCALE_SPACE, inputImage: imageData,
  numberOfOctaves: 3, scalesPerOctave: 3, minBlurLevel: 0.8, assumedBlur: 0.5, chunkSize: 32 } });
const wss = posted[posted.length - 1].scaleSpace;
onmessage({ data: { type: sift.WorkerMessageTypes.COMPUTE_DIFFERENCE_OF_GAUSSIANS, scaleSpace: wss } });
const wdd = posted[posted.length - 1].differenceOfGaussians;
onmessage({ data: { type: sift.WorkerMessageTypes.FIND_CANDIDATE_KEYPOINTS, differenceOfGaussians: wdd,
  octaveBaseImages: wss.map(o => o[0].image), scalesPerOctave: 3 } });
const cc = posted[posted.length - 1].candidateKeypoints;
let nc = 0;
cc.forEach(o => o.forEach(s => { nc += s.localExtremas.length; }));
out.worker = {
  types: posted.map(m => m.type), candidates: nc,
  lowMarkers: posted.filter(m => m.type === 'received-candidate-keypoint-marker' && m.isLowContrast).length,
  firstGaussPreview: (() => { const m = posted[0]; return { octave: m.octave, w: m.imageData.width, h: m.imageData.height,
    px: Array.from(m.imageData.data.subarray(0, 16)) }; })(),
};
out.gaussPlane00 = Array.from(wss[0][0].image[0].slice(0, 4));
fs.writeFileSync(outPath, JSON.stringify(out));
