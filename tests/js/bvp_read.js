// Reads a BVP archive through ReaderFactory('bvp') + Volume.load() (host
// assembly, WebGPUVolume.readModality's placement loop) and writes the volume.
// Usage: node bvp_read.js <in.bvp> <out.raw>
'use strict';
const fs = require('fs');
const path = require('path');
const V = require(path.join(__dirname, '..', '..', 'vpt-spectral-volume-rendering_amd', 'js'));

(async () => {
  const reader = new (V.ReaderFactory('bvp'))(new V.FileLoader(process.argv[2]));
  const volume = new V.Volume(reader);
  await volume.load();
  const h = volume.hostVolume;
  const zip = new V.ZIPReader(new V.BufferLoader(fs.readFileSync(process.argv[2])));
  const files = await zip.getFiles();
  fs.writeFileSync(process.argv[3], Buffer.from(h.data.buffer, h.data.byteOffset, h.data.length));
  console.log(JSON.stringify({ width: h.width, height: h.height, depth: h.depth, files: files.length }));
})().catch(e => { console.error(e.stack); process.exit(1); });
