#!/usr/bin/env node
// Generates the golden fixtures in tests/golden/ by RUNNING THE REFERENCE'S
// OWN JS in this container (Node 12). Never run on the GPU box: it reads
// /root/reference, which exists only here. Outputs are committed.
//
//   cie1931.json          CIE_SPECTRUM of src/js/utils/Spectrum.js:12-19
//                         (imported as an ES module from a /tmp copy)
//   spectrum_buffers.json the 64-f32 spectrum buffer the reference uploads
//                         (WebGPUMCMSpectralComputeRenderer.js:311-312), with
//                         x/y/z coefficients produced by the reference's own
//                         compute_spectral_coefficients (js:379-412), extracted
//                         from the file text and evaluated, for the bin layouts
//                         the reference names (js:77-79) plus two more.
//   mvp_inverse.json      Float32 bits of invert(P*V*M) computed with the
//                         reference's vendored gl-matrix 3.4.1
//                         (src/lib/gl-matrix-min.js) following
//                         _renderFrame js:266-274, Transform.js:64-70 and
//                         PerspectiveCamera.js:9-17, for the default camera
//                         (WebGPURenderingContext.js:37-39) and other poses.
//
// Usage: node tests/golden/make_golden.js [/root/reference]
'use strict';
const fs = require('fs');
const path = require('path');
const os = require('os');

const REF = process.argv[2] || '/root/reference';
const OUT = __dirname;

function f32bits(x) {
  const b = new ArrayBuffer(4);
  new Float32Array(b)[0] = x;
  return new Uint32Array(b)[0];
}

async function main() {
  // --- CIE table: import the reference module as ESM from a temp copy.
  const specSrc = fs.readFileSync(path.join(REF, 'src/js/utils/Spectrum.js'), 'utf8');
  const tmp = fs.mkdtempSync(path.join(os.tmpdir(), 'vptgold-'));
  const specMjs = path.join(tmp, 'Spectrum.mjs');
  fs.writeFileSync(specMjs, specSrc);
  const specMod = await import(specMjs);
  const CIE = specMod.CIE_SPECTRUM;
  fs.writeFileSync(path.join(OUT, 'cie1931.json'), JSON.stringify({
    source: 'reference src/js/utils/Spectrum.js:12-19 (CIE 1931 2deg, 1 nm), imported by make_golden.js',
    first_wavelength: CIE.first_wavelenght, step: CIE.step, length: CIE.length,
    X: Array.from(CIE.X), Y: Array.from(CIE.Y), Z: Array.from(CIE.Z),
  }) + '\n');

  // --- compute_spectral_coefficients: the method body, evaluated as is.
  const rendSrc = fs.readFileSync(
    path.join(REF, 'src/js/renderers/WebGPUMCMSpectralComputeRenderer.js'), 'utf8');
  const m = rendSrc.match(/\ncompute_spectral_coefficients\(\)\s*\{([\s\S]*?)\n\}\n/);
  if (!m) throw new Error('compute_spectral_coefficients not found');
  const method = new Function('CIE_SPECTRUM', m[1]);
  const layouts = {
    '12': [400, 425, 450, 475, 500, 525, 550, 575, 600, 625, 650, 675, 700], // js:79
    '6': [400, 450, 500, 550, 600, 650, 700],                              // js:78
    '3': [400, 500, 600, 700],                                             // js:77
    '8_uneven': [380, 410, 440, 470, 520, 560, 610, 660, 780],
    '12_wide': [360, 395, 430, 465, 500, 535, 570, 605, 640, 675, 710, 745, 780],
  };
  const buffers = {};
  for (const [name, bins] of Object.entries(layouts)) {
    const self = { n_bins: bins.length - 1, spectrumRepresentationData: bins };
    method.call(self, CIE);
    // js:311-312 — Float32Array([n_bins, ...bins, ...x, ...y, ...z]) into a 256-B buffer
    const arr = new Float32Array(64);
    arr.set([self.n_bins, ...bins, ...self.x_coeff, ...self.y_coeff, ...self.z_coeff]);
    buffers[name] = {
      bins, n_bins: self.n_bins,
      x_coeff: self.x_coeff, y_coeff: self.y_coeff, z_coeff: self.z_coeff,
      buffer_bits: Array.from(arr, f32bits),
    };
  }
  fs.writeFileSync(path.join(OUT, 'spectrum_buffers.json'), JSON.stringify({
    source: 'reference WebGPUMCMSpectralComputeRenderer.js compute_spectral_coefficients (js:379-412) run on Spectrum.js',
    layouts: buffers,
  }, null, 1) + '\n');

  // --- mvpInverse with the vendored gl-matrix.
  const glm = require(path.join(REF, 'src/lib/gl-matrix-min.js'));
  const { mat4, quat, vec3 } = glm;
  function inverseLocalMatrix(translation, rotation, scale) { // Transform.js:64-70
    const inverseScale = vec3.inverse(vec3.create(), scale);
    const inverseRotation = quat.invert(quat.create(), rotation);
    const inverseTranslation = vec3.negate(vec3.create(), translation);
    const matrix = mat4.create();
    mat4.scale(matrix, matrix, inverseScale);
    mat4.multiply(matrix, matrix, mat4.fromQuat(mat4.create(), inverseRotation));
    mat4.translate(matrix, matrix, inverseTranslation);
    return matrix;
  }
  function mvpInverse(cam) { // js:266-274
    const modelMatrix = mat4.fromTranslation(mat4.create(), [-0.5, -0.5, -0.5]);
    const viewMatrix = inverseLocalMatrix(cam.translation, cam.rotation, [1, 1, 1]);
    const projectionMatrix = mat4.perspective(mat4.create(), cam.fovy, cam.aspect, 0.1, 100);
    const matrix = mat4.create();
    mat4.multiply(matrix, modelMatrix, matrix);
    mat4.multiply(matrix, viewMatrix, matrix);
    mat4.multiply(matrix, projectionMatrix, matrix);
    mat4.invert(matrix, matrix);
    return matrix;
  }
  const rotY = quat.setAxisAngle(quat.create(), [0, 1, 0], 0.6);
  const rotXY = quat.multiply(quat.create(), quat.setAxisAngle(quat.create(), [1, 0, 0], -0.4), rotY);
  const cams = {
    default: { translation: [0, 0, 2], rotation: [0, 0, 0, 1], fovy: 1, aspect: 1 },
    near: { translation: [0.1, -0.05, 1.3], rotation: [0, 0, 0, 1], fovy: 1, aspect: 1 },
    orbit: { translation: [1.13, 0.0, 1.65], rotation: Array.from(rotY), fovy: 1, aspect: 1 },
    orbit_tilted: { translation: [1.0, -0.8, 1.5], rotation: Array.from(rotXY), fovy: 0.8, aspect: 1 },
  };
  const mvps = {};
  for (const [name, cam] of Object.entries(cams)) {
    mvps[name] = { camera: cam, bits: Array.from(mvpInverse(cam), f32bits) };
  }
  fs.writeFileSync(path.join(OUT, 'mvp_inverse.json'), JSON.stringify({
    source: 'reference src/lib/gl-matrix-min.js 3.4.1, sequence of WebGPUMCMSpectralComputeRenderer.js:266-274',
    cameras: mvps,
  }, null, 1) + '\n');

  fs.rmSync ? fs.rmSync(tmp, { recursive: true }) : fs.rmdirSync(tmp, { recursive: true });
  console.log('golden fixtures written to', OUT);
}

main().catch(e => { console.error(e); process.exit(1); });
