// The drop-in JS host timed end to end (bench.py's `js_api` line): Node drives
// MCMSpectralComputeRenderer exactly as the reference application drives
// WebGPUMCMSpectralComputeRenderer (WebGPURenderingContext.js:187: one
// renderer.render() per frame), through the N-API shim and the C-ABI into the
// HIP march. Every render() re-sends the unchanged uniforms (js:295-309), as the
// reference does; the library queues the passes into fused launches.
//
//   node tools/js_render_bench.js <case.json>   -> one JSON line on stdout
// case: { R, volume_path, W, H, D, tf_path, spectrum_path, extinction, steps,
//         settle_ms, warmup, passes }
'use strict';
const fs = require('fs');
const path = require('path');

const ROOT = path.resolve(__dirname, '..');
const V = require(path.join(ROOT, 'vpt-spectral-volume-rendering_amd', 'js'));

(async () => {
  const c = JSON.parse(fs.readFileSync(process.argv[2]));
  const spec = new Float32Array(new Uint8Array(fs.readFileSync(c.spectrum_path)).buffer);
  const renderer = new V.MCMSpectralComputeRenderer(V.createDevice(0), null, new V.Camera({}), null,
    { resolution: c.R, spectrumBuffer: spec });
  renderer.setMaterialTransferFunction(new Uint8Array(fs.readFileSync(c.tf_path)), false);
  renderer.extinction = c.extinction;
  renderer.bounces = 8;
  renderer.steps = c.steps;
  const volume = new V.Volume(new V.RAWReader(new V.FileLoader(c.volume_path),
    { width: c.W, height: c.H, depth: c.D }));
  await renderer.loadVolume(volume);             // block-wise HBM ingest, then reset()

  const now = () => Number(process.hrtime.bigint()) / 1e6;  // ms
  // clock settling (the engine clock ramps over the first ~30 ms of load), then warm-up
  const t = now();
  while (now() - t < c.settle_ms) {
    for (let k = 0; k < 256; k++) renderer.render();
    renderer.synchronize();
  }
  for (let k = 0; k < c.warmup; k++) renderer.render();
  renderer.synchronize();

  const l0 = renderer.lastLaunch().launches;
  const t0 = now();
  for (let k = 0; k < c.passes; k++) renderer.render();
  renderer.synchronize();
  const ms = now() - t0;
  const launches = renderer.lastLaunch().launches - l0;
  renderer.destroy();
  const steps = c.R * c.R * c.steps * c.passes;
  console.log(JSON.stringify({ value: steps / (ms * 1e-3) / 1e6, ms_per_step: ms / c.passes,
    steps: c.passes, launches, node: process.version }));
})().catch(e => { console.error(e.stack); process.exit(1); });
