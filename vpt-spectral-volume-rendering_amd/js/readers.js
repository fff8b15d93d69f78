'use strict';
// Volume ingest, mirroring the reference's reader/volume pipeline:
//   RAWReader.readMetadata / readBlock  (readers/RAWReader.js:15-70): one
//     'default' modality, one z-slice block per placement;
//   Volume.readModality  (WebGPUVolume.js:34-96): for every placement, read
//     its block and write it at its origin — here into the renderer's HBM
//     volume through vptmcm_volume_write_block instead of queue.writeTexture.
//   ZIPReader / BVPReader (readers/ZIPReader.js:20-91, BVPReader.js:13-29): the
//     zip central directory, and a BVP's manifest.json + per-block files;
//   ReaderFactory (readers/ReaderFactory.js): 'bvp' | 'raw' | 'zip'.
// Loaders return Uint8Array ranges (AjaxLoader/BlobLoader's readData) and the
// total length (readLength, AbstractLoader.js).
const fs = require('fs');
const zlib = require('zlib');

class BufferLoader {
  constructor(bytes) {
    this.bytes = bytes instanceof Uint8Array ? bytes : new Uint8Array(bytes);
  }

  async readLength() {
    return this.bytes.length;
  }

  async readData(start, end) {
    return this.bytes.subarray(start, end);
  }
}

class FileLoader {
  constructor(path) {
    this.path = path;
  }

  async readLength() {
    return fs.statSync(this.path).size;
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

// ZIP archive reader (ZIPReader.js): end-of-central-directory record, central
// directory entries, local header -> file data. The reference returns the
// stored bytes as they are (BVP archives are written uncompressed, method 0);
// deflated entries (method 8) are inflated here with Node's zlib.
class ZIPReader {
  constructor(loader) {
    this._loader = loader;
    this._eocd = null;
    this._cd = null;
  }

  async getFiles() {
    if (!this._cd) await this._readCD();
    return this._cd.map(e => e.name);
  }

  async readFile(fileName) {
    if (!this._cd) await this._readCD();
    const entry = this._cd.find(e => e.name === fileName);
    if (!entry) throw new Error(`ZIPReader: file ${fileName} not in CD`);
    const headerStart = entry.headerOffset;
    const headerEnd = headerStart + 30;
    const header = view(await this._loader.readData(headerStart, headerEnd));
    if (header.getUint32(0, true) !== 0x04034b50) throw new Error(`ZIPReader: bad local header for ${fileName}`);
    const dataStart = headerEnd + header.getUint16(26, true) + header.getUint16(28, true);
    const data = await this._loader.readData(dataStart, dataStart + entry.compressedSize);
    if (entry.method === 0) return data;
    if (entry.method === 8) return new Uint8Array(zlib.inflateRawSync(Buffer.from(data)));
    throw new Error(`ZIPReader: unsupported compression method ${entry.method} for ${fileName}`);
  }

  async _readEOCD() {
    const MIN_EOCD_SIZE = 22;
    const length = await this._loader.readLength();
    const offset = Math.max(length - MIN_EOCD_SIZE, 0);
    const v = view(await this._loader.readData(offset, offset + Math.min(length, MIN_EOCD_SIZE)));
    if (v.byteLength < MIN_EOCD_SIZE || v.getUint32(0, true) !== 0x06054b50) {
      throw new Error('ZIPReader: no end-of-central-directory record (archive comments are not supported)');
    }
    this._eocd = { entries: v.getUint16(10, true), size: v.getUint32(12, true), offset: v.getUint32(16, true) };
  }

  async _readCD() {
    if (!this._eocd) await this._readEOCD();
    const { offset: cdStart, size, entries: n } = this._eocd;
    const bytes = await this._loader.readData(cdStart, cdStart + size);
    const v = view(bytes);
    const entries = [];
    let o = 0;
    for (let i = 0; i < n; i++) {
      if (v.getUint32(o, true) !== 0x02014b50) throw new Error('ZIPReader: corrupt central directory');
      const nameLength = v.getUint16(o + 28, true);
      entries.push({
        gpflag: v.getUint16(o + 8, true),
        method: v.getUint16(o + 10, true),
        compressedSize: v.getUint32(o + 20, true),
        uncompressedSize: v.getUint32(o + 24, true),
        name: Buffer.from(bytes.buffer, bytes.byteOffset + o + 46, nameLength).toString('utf8'),
        headerOffset: v.getUint32(o + 42, true),
      });
      o += 46 + nameLength + v.getUint16(o + 30, true) + v.getUint16(o + 32, true);
    }
    this._cd = entries;
  }
}

function view(u8) {
  return new DataView(u8.buffer, u8.byteOffset, u8.byteLength);
}

// BVP volume archive (BVPReader.js): manifest.json holds modalities (dimensions,
// placements) and blocks (url, dimensions); each block is a file in the zip.
class BVPReader {
  constructor(loader) {
    this._loader = loader;
    this._metadata = null;
    this._zipReader = new ZIPReader(loader);
  }

  async readMetadata() {
    const data = await this._zipReader.readFile('manifest.json');
    this._metadata = JSON.parse(Buffer.from(data.buffer, data.byteOffset, data.byteLength).toString('utf8'));
    return this._metadata;
  }

  async readBlock(block) {
    if (!this._metadata) await this.readMetadata();
    return this._zipReader.readFile(this._metadata.blocks[block].url);
  }
}

function ReaderFactory(which) {  // readers/ReaderFactory.js
  switch (which) {
    case 'bvp': return BVPReader;
    case 'raw': return RAWReader;
    case 'zip': return ZIPReader;
    default: throw new Error('No suitable class');
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

module.exports = { BufferLoader, FileLoader, RAWReader, ZIPReader, BVPReader, ReaderFactory, Volume };
