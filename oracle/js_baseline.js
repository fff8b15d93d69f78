'use strict';
// js_baseline.js — TEST INFRASTRUCTURE ONLY: runs oracle/mcm_march.js (the
// scalar JavaScript re-execution of the march) over worker_threads, rows
// interleaved over the workers, every buffer in shared memory.
//
//   node oracle/js_baseline.js <dir> check <threads>
//       reset with seeds[0], one pass per further seed; writes photons.bin,
//       rgb32.bin and rgba16.bin (the last pass) into <dir>
//   node oracle/js_baseline.js <dir> bench <threads> <seconds>
//       reset, one warm-up pass, then passes until <seconds> have elapsed;
//       prints one JSON line {passes, seconds, threads, host_cpus, ...}
//
// <dir>/meta.json: {R, W, H, D, mvp_bits[16], inv_res_bits[2], blur_bits,
// extinction_bits, max_bounces, steps, light_dir_bits[3], seeds[]} (f32 values
// as their bit patterns); vol.bin (u8 W*H*D, x fastest), tf.bin (u8 256*256*4),
// light.bin (u8 256), spec.bin (f32 64).
const fs = require('fs');
const os = require('os');
const path = require('path');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const { March } = require('./mcm_march.js');

function f32(bits) {
  const u = new Uint32Array([bits >>> 0]);
  return new Float32Array(u.buffer)[0];
}

function uniforms(meta, seed) {
  return {
    mvp: Float32Array.from(meta.mvp_bits.map(f32)),
    invRes: Float32Array.from(meta.inv_res_bits.map(f32)),
    blur: f32(meta.blur_bits),
    extinction: f32(meta.extinction_bits),
    maxBounces: meta.max_bounces,
    steps: meta.steps,
    lightDir: Float32Array.from(meta.light_dir_bits.map(f32)),
    seedBits: seed >>> 0,
  };
}

function shared(bytes, src) {
  const sab = new SharedArrayBuffer(bytes);
  if (src) new Uint8Array(sab).set(new Uint8Array(src.buffer, src.byteOffset, bytes));
  return sab;
}

if (!isMainThread) {
  const d = workerData;
  const m = new March({
    R: d.meta.R, W: d.meta.W, H: d.meta.H, D: d.meta.D,
    vol: new Uint8Array(d.vol), tf: new Uint8Array(d.tf), light: new Uint8Array(d.light),
    spec: new Float32Array(d.spec), photons: d.photons, u: uniforms(d.meta, 0),
  });
  const rgb32 = new Float32Array(d.rgb32);
  const rgba16 = new Uint16Array(d.rgba16);
  const R = d.meta.R;
  parentPort.on('message', (msg) => {
    m.u.seedBits = msg.seed >>> 0;
    for (let y = d.id; y < R; y += d.n) {
      if (msg.op === 'reset') m.resetRows(y, y + 1);
      else m.renderRows(y, y + 1, rgb32, rgba16);
    }
    parentPort.postMessage('done');
  });
} else {
  const [dir, mode, threadsArg, secondsArg] = process.argv.slice(2);
  const meta = JSON.parse(fs.readFileSync(path.join(dir, 'meta.json'), 'utf8'));
  const R = meta.R;
  const n = Math.max(1, Math.min(parseInt(threadsArg || '1', 10), R));
  const rd = (f) => fs.readFileSync(path.join(dir, f));
  const bufs = {
    vol: shared(meta.W * meta.H * meta.D, rd('vol.bin')),
    tf: shared(256 * 256 * 4, rd('tf.bin')),
    light: shared(256, rd('light.bin')),
    spec: shared(64 * 4, rd('spec.bin')),
    photons: shared(R * R * 144),
    rgb32: shared(R * R * 12),
    rgba16: shared(R * R * 8),
  };
  const workers = [];
  for (let id = 0; id < n; id++) workers.push(new Worker(__filename, { workerData: { ...bufs, meta, id, n } }));
  const all = (op, seed) => Promise.all(workers.map((w) => new Promise((res) => {
    w.once('message', res);
    w.postMessage({ op, seed });
  })));

  (async () => {
    const seeds = meta.seeds;
    await all('reset', seeds[0]);
    if (mode === 'check') {
      for (let k = 1; k < seeds.length; k++) await all('render', seeds[k]);
      fs.writeFileSync(path.join(dir, 'photons.bin'), Buffer.from(bufs.photons));
      fs.writeFileSync(path.join(dir, 'rgb32.bin'), Buffer.from(bufs.rgb32));
      fs.writeFileSync(path.join(dir, 'rgba16.bin'), Buffer.from(bufs.rgba16));
    } else {
      const budget = parseFloat(secondsArg || '10');
      await all('render', seeds[1]);  // warm-up pass (JIT)
      let passes = 0;
      const t0 = process.hrtime.bigint();
      let el = 0;
      while (el < budget) {
        await all('render', seeds[2 + (passes % (seeds.length - 2))]);
        passes++;
        el = Number(process.hrtime.bigint() - t0) * 1e-9;
      }
      console.log(JSON.stringify({ passes, seconds: el, threads: n, host_cpus: os.cpus().length,
        photon_steps_per_s: R * R * meta.steps * passes / el, node: process.version }));
    }
    workers.forEach((w) => w.terminate());
  })();
}
