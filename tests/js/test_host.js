// CPU tests of the JavaScript host (no GPU): camera math and spectrum buffers
// against the goldens produced by the reference's own JS, the property/event
// surface, the factory, the RAW reader + volume assembly, and that the N-API
// addon loads and fails loudly without a device. Exit code 0 = pass.
'use strict';
const assert = require('assert');
const fs = require('fs');
const path = require('path');

const ROOT = path.resolve(__dirname, '..', '..');
const V = require(path.join(ROOT, 'vpt-spectral-volume-rendering_amd', 'js'));
const gold = f => JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', f)));

const tests = [];
const test = (name, fn) => tests.push([name, fn]);

test('mvpInverse bits equal the reference gl-matrix', () => {
  for (const [name, c] of Object.entries(gold('mvp_inverse.json').cameras)) {
    const cam = new V.Camera({ translation: c.camera.translation, rotation: c.camera.rotation,
      fovy: c.camera.fovy, aspect: c.camera.aspect });
    const bits = Array.from(new Uint32Array(V.mvpInverse(cam).buffer));
    assert.deepStrictEqual(bits, c.bits, name);
  }
});

test('spectrum buffers equal the reference compute_spectral_coefficients', () => {
  const cie = gold('cie1931.json');
  for (const [name, l] of Object.entries(gold('spectrum_buffers.json').layouts)) {
    const c = V.spectrum.computeSpectralCoefficients(l.bins, cie);
    const buf = V.spectrum.packSpectrumBuffer(l.bins, c);
    assert.deepStrictEqual(Array.from(new Uint32Array(buf.buffer)), l.buffer_bits, name);
  }
  assert.throws(() => V.spectrum.packSpectrumBuffer(new Array(15).fill(400), { x: [], y: [], z: [] }),
    /12/);
});

test('UI models: material TF painting (MaterialTransferFunction.js semantics)', () => {
  const m = new V.MaterialTransferFunctionModel();
  assert.strictEqual(m.materials.length, 1);
  assert.ok(m.materials[0].albedo.every(v => v === 127), 'default material is 127 everywhere');
  assert.ok(m.value.every(v => v === 0), 'the TF starts empty');
  let changes = 0;
  m.addEventListener('change', () => changes++);
  const col = Uint8Array.from({ length: 256 }, (_, c) => (60 + c * 0.7) | 0);
  const a = m.addMaterial(180, 60, col);
  m.paint(90, 20, a.id);  // reversed range, rows 20..90
  assert.strictEqual(changes, 1);
  const tx = (r, c) => Array.from(m.value.subarray((r * 256 + c) * 4, (r * 256 + c) * 4 + 4));
  assert.deepStrictEqual(tx(20, 0), [180, 60, 60, 0]);
  assert.deepStrictEqual(tx(90, 255), [180, 60, col[255], 0]);
  assert.deepStrictEqual(tx(19, 7), [0, 0, 0, 0]);
  assert.deepStrictEqual(tx(91, 7), [0, 0, 0, 0]);
  m.paint(50, 60, a.id, true);  // erase
  assert.deepStrictEqual(tx(55, 3), [0, 0, 0, 0]);
  assert.deepStrictEqual(tx(49, 3), [180, 60, col[3], 0]);
  m.paint(-5, 300, m.materials[0].id);  // clamped to the canvas
  assert.deepStrictEqual(tx(0, 0), [127, 127, 127, 0]);
  assert.deepStrictEqual(tx(255, 255), [127, 127, 127, 0]);
  assert.strictEqual(m.removeMaterial(a.id), true);
  assert.strictEqual(m.removeMaterial(m.materials[0].id), false, 'the last material stays');
});

test('UI models: spectrum markers (SpectrumRepresentation.js semantics)', () => {
  const s = new V.SpectrumRepresentationModel();
  // the default (12 bins, k = 0) is the renderer's default bin layout (js:79)
  assert.deepStrictEqual(s.getBins(), gold('spectrum_buffers.json').layouts['12'].bins);
  s.arrange(0, 6);
  assert.deepStrictEqual(s.getBins(), gold('spectrum_buffers.json').layouts['6'].bins);
  s.arrange(2, 8);  // exponential spacing: denser at the blue end, whole nm, sorted
  const b = s.getBins();
  assert.strictEqual(b.length, 9);
  assert.strictEqual(b[0], 400);
  assert.strictEqual(b[8], 700);
  for (let i = 1; i < 9; i++) assert.ok(b[i] > b[i - 1]);
  for (let i = 2; i < 9; i++) assert.ok(b[i] - b[i - 1] >= b[i - 1] - b[i - 2] - 1);
  const x3 = (Math.exp(2 * 3 / 8) - 1) / (Math.exp(2) - 1);
  assert.strictEqual(b[3], Math.round(400 + 300 * x3));
  s.moveMarker(8, 1.7);  // clamped to the track
  assert.strictEqual(s.getBins()[8], 700);
  s.moveMarker(0, 0.5);  // crossing markers are re-sorted
  const c = s.getBins();
  assert.ok(c.every((v, i) => i === 0 || v >= c[i - 1]));
});

test('UI models drive a renderer like the element listeners', () => {
  const calls = [];
  const fake = {
    setLight: (spd, dir) => calls.push(['light', spd[0], Array.from(dir)]),
    setSpectrumRepresentation: bins => calls.push(['bins', bins.length]),
    setMaterialTransferFunction: v => calls.push(['tf', v.length]),
  };
  const le = new V.LightEditorModel(), sr = new V.SpectrumRepresentationModel(),
    tf = new V.MaterialTransferFunctionModel();
  V.connectUiModels(fake, { lightEditor: le, spectrumRepresentation: sr, materialTransferFunction: tf });
  assert.deepStrictEqual(calls, [['light', 100, [1, 0, 0]], ['bins', 13], ['tf', 262144]]);
  le.setDirection([0, 1, 0]);
  sr.arrange(0, 3);
  tf.paint(0, 10);
  assert.deepStrictEqual(calls.slice(3), [['light', 100, [0, 1, 0]], ['bins', 4], ['tf', 262144]]);
  assert.throws(() => le.setSpectrum(new Uint8Array(10)), /256/);
});

test('property bag + change events', () => {
  const bag = new V.PropertyBag();
  bag.registerProperties([{ name: 'extinction', value: 1 }, { name: 'steps', value: 8 }]);
  assert.strictEqual(bag.extinction, 1);
  const seen = [];
  bag.addEventListener('change', e => seen.push(e.detail.name));
  bag.setProperty('extinction', 32);
  assert.strictEqual(bag.extinction, 32);
  assert.deepStrictEqual(seen, ['extinction']);
});

test('factory', () => {
  assert.strictEqual(V.RendererFactory('mcm-spectral-compute'), V.MCMSpectralComputeRenderer);
  assert.throws(() => V.RendererFactory('mip'), /No suitable class/);
});

test('RAW reader placements and volume assembly', async () => {
  const W = 5, H = 4, D = 3;
  const bytes = new Uint8Array(W * H * D).map((_, i) => (i * 7) & 255);
  const reader = new V.RAWReader(new V.BufferLoader(bytes), { width: W, height: H, depth: D });
  const meta = await reader.readMetadata();
  assert.strictEqual(meta.modalities[0].placements.length, D);
  assert.deepStrictEqual(meta.modalities[0].placements[2].position, { x: 0, y: 0, z: 2 });
  const vol = new V.Volume(reader);
  await vol.load();
  assert.deepStrictEqual(Array.from(vol.hostVolume.data), Array.from(bytes));
  await assert.rejects(vol.readModality('nope', { begin() {}, block() {}, end() {} }), /does not exist/);
});

test('addon loads; renderer construction fails loudly without a GPU', () => {
  const A = V.native();
  for (const f of ['create', 'destroy', 'setVolume', 'volumeBegin', 'volumeWriteBlock', 'volumeEnd',
    'setMaterialTF', 'setLight', 'setSpectrum', 'setParams', 'reset', 'render', 'renderPasses',
    'synchronize', 'readRGBA16F', 'readPhotons', 'writePhotons', 'enableKernelTiming', 'kernelTime',
    'commUniqueId', 'commInit', 'commAllreduceRadiance', 'commReadComposite', 'commBarrier', 'setBand', 'commGatherBands', 'version',
    'tonemapArtistic', 'readRGB', 'lastLaunch', 'composite', 'readComposite', 'groupDevices', 'setMacroSkip']) {
    assert.strictEqual(typeof A[f], 'function', f);
  }
  assert.ok(/gfx950/.test(A.version()));
  let haveGpu = false;
  try { A.destroy(A.create(16, -1, 1)); haveGpu = true; } catch (e) { haveGpu = false; }
  if (haveGpu) return;  // on a GPU box the no-device path cannot be exercised
  assert.throws(() => new V.MCMSpectralComputeRenderer(V.createDevice(0), null, new V.Camera(), null,
    { resolution: 16, cie: gold('cie1931.json') }), e => e.vptmcmCode === -2 && /HIP device/.test(e.message));
  assert.throws(() => A.create(0, -1, 1), /resolution/);
  // device lists: validated in the shim / the JS class before any device call
  assert.throws(() => A.create(16, -1, 1, 0, []), /1 to VPTMCM_MAX_DEVICES/);
  assert.throws(() => A.create(16, -1, 1, 0, [0, 1, 2, 3, 4, 5, 6, 7, 8]), /1 to VPTMCM_MAX_DEVICES/);
  assert.throws(() => A.create(16, -1, 1, 0, ['x']), /integer ordinals/);
  assert.throws(() => new V.MCMSpectralComputeRenderer(V.createDevice([0, 1], 'corner8', 'nccl'), null,
    new V.Camera(), null, { resolution: 16, cie: gold('cie1931.json') }), /unknown transport/);
  assert.throws(() => new V.MCMSpectralComputeRenderer({ devices: [] }, null, new V.Camera(), null,
    { resolution: 16, cie: gold('cie1931.json') }), /1 to 8 device ordinals/);
  // a valid list reaches the library, which fails loudly without a device
  assert.throws(() => new V.MCMSpectralComputeRenderer(V.createDevice([0, 1]), null, new V.Camera(), null,
    { resolution: 16, cie: gold('cie1931.json') }), e => e.vptmcmCode === -2 && /HIP device/.test(e.message));
});

test('createDevice: an ordinal or a device list', () => {
  assert.deepStrictEqual(V.createDevice(3), { ordinal: 3, layout: 'column4' });
  assert.deepStrictEqual(V.createDevice([0, 1, 2], 'brick8'), { devices: [0, 1, 2], layout: 'brick8', transport: 'peer' });
  assert.deepStrictEqual(V.createDevice([4, 5], 'corner8', 'rccl').transport, 'rccl');
});

test('tone mapper surface mirrors WebGPUArtisticToneMapper (properties, factory)', () => {
  const tm = new (V.ToneMapperFactory('artistic'))(V.createDevice(0), null, null, { resolution: 8 });
  const byName = {};
  for (const p of tm.properties) byName[p.name] = p;
  assert.deepStrictEqual(Object.keys(byName), ['low', 'high', 'mid', 'saturation', 'gamma']);
  assert.strictEqual(tm.low, 0);
  assert.strictEqual(tm.high, 1);
  assert.strictEqual(tm.mid, 0.5);
  assert.strictEqual(tm.saturation, 1);
  assert.strictEqual(tm.gamma, 2.2);
  assert.strictEqual(byName.mid.min, 0.00001);
  assert.strictEqual(tm.getTexture(), null);
  assert.throws(() => tm.render(), /no texture/);
  assert.throws(() => tm.setTexture(new Uint16Array(4)), /HIP renderer/);
  assert.throws(() => V.ToneMapperFactory('reinhard'), /No suitable class/);
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try {
      await fn();
      console.log(`ok   ${name}`);
    } catch (e) {
      failed++;
      console.log(`FAIL ${name}: ${e.stack}`);
    }
  }
  process.exit(failed ? 1 : 0);
})();
