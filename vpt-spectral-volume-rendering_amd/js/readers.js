'use strict';
// Volume ingest, mirroring the reference's reader/volume pipeline:
//   RAWReader.readMetadata / readBlock  (readers/RAWReader.js:15-70): one
//     'default' modality, one z-slice block per placement;
//   Volume.readModality  (WebGPUVolume.js:34-96): for every placement, read
//     its block and write it at its origin — here into the renderer's HBM
//     volume through vptmcm_volume_write_block instead of queue.writeTexture.
// Loaders return Uint8Array ranges (AjaxLoader/BlobLoader's readData).
const fs = require('fs');

class BufferLoader {
  constructor(bytes) {
    this.bytes = bytes instanceof Uint8Array ? bytes : new Uint8Array(bytes);
  }

  async readData(start, end) {
    return this.bytes.subarray(start, end);
  }
}

class FileLoader {
  constructor(path) {
    this.path = path;
  }

  async readData(start, end) {
    const fd = fs.openSync(this.path, 'r');
    try {
      const out = Buffer.alloc(end - start);
      fs.readSync(fd, out, 0, end - start, start);
      return new Uint8Array(out.buffer, out.byteOffset, out.length);
    } finally {
      fs.closeSync(fd);
    }
  }
}

class RAWReader {
  constructor(loader, options = {}) {
    this._loader = loader;
    this.width = options.width || 0;
    this.height = options.height || 0;
    this.depth = options.depth || 0;
  }

  async readMetadata() {
    const modality = {
      name: 'default',
      dimensions: { width: this.width, height: this.height, depth: this.depth },
      transform: { matrix: [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1] },
      format: 6403, internalFormat: 33321, type: 5121,  // RED, R8, UNSIGNED_BYTE
      placements: [],
    };
    const metadata = { meta: { version: 1 }, modalities: [modality], blocks: [] };
    for (let z = 0; z < this.depth; z++) {
      modality.placements.push({ index: z, position: { x: 0, y: 0, z } });
      metadata.blocks.push({ url: 'default', format: 'raw',
        dimensions: { width: this.width, height: this.height, depth: 1 } });
    }
    return metadata;
  }

  async readBlock(block) {
    const slice = this.width * this.height;
    return this._loader.readData(block * slice, (block + 1) * slice);
  }
}

class Volume {
  constructor(reader) {
    this._reader = reader;
    this.metadata = null;
    this.modality = null;
    this.ready = false;
    this._sinks = [];
  }

  async readMetadata() {
    if (!this.metadata) this.metadata = await this._reader.readMetadata();
    return this.metadata;
  }

  // Stream every block of a modality into `sink` ({begin, block, end}).
  async readModality(modalityName, sink) {
    this.ready = false;
    await this.readMetadata();
    const modality = this.metadata.modalities.find(m => m.name === modalityName);
    if (!modality) throw new Error(`Modality '${modalityName}' does not exist`);
    this.modality = modality;
    const { width, height, depth } = modality.dimensions;
    sink.begin(width, height, depth);
    for (const { index, position } of modality.placements) {
      const data = await this._reader.readBlock(index);
      const dims = this.metadata.blocks[index].dimensions;
      sink.block(new Uint8Array(data), position.x, position.y, position.z,
        dims.width, dims.height, dims.depth);
    }
    sink.end();
    this.ready = true;
  }

  // With a sink, stream the blocks (e.g. into HBM); without one, assemble the
  // host copy `hostVolume` = { data, width, height, depth } (the texture content).
  async load(sink) {
    if (sink) {
      await this.readModality('default', sink);
      return;
    }
    let host = null;
    await this.readModality('default', {
      begin: (width, height, depth) => {
        host = { data: new Uint8Array(width * height * depth), width, height, depth };
      },
      block: (data, x, y, z, w, h, d) => {
        for (let k = 0; k < d; k++) {
          for (let j = 0; j < h; j++) {
            const src = (k * h + j) * w;
            const dst = ((z + k) * host.height + (y + j)) * host.width + x;
            host.data.set(data.subarray(src, src + w), dst);
          }
        }
      },
      end: () => {},
    });
    this.hostVolume = host;
  }
}

module.exports = { BufferLoader, FileLoader, RAWReader, Volume };
