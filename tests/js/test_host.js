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
    'commUniqueId', 'commInit', 'commAllreduceRadiance', 'commReadComposite', 'commBarrier', 'version',
    'tonemapArtistic']) {
    assert.strictEqual(typeof A[f], 'function', f);
  }
  assert.ok(/gfx950/.test(A.version()));
  let haveGpu = false;
  try { A.destroy(A.create(16, -1, 1)); haveGpu = true; } catch (e) { haveGpu = false; }
  if (haveGpu) return;  // on a GPU box the no-device path cannot be exercised
  assert.throws(() => new V.MCMSpectralComputeRenderer(V.createDevice(0), null, new V.Camera(), null,
    { resolution: 16, cie: gold('cie1931.json') }), e => e.vptmcmCode === -2 && /HIP device/.test(e.message));
  assert.throws(() => A.create(0, -1, 1), /resolution/);
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
