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

// ZIP archive reader, the ZIPReader.js surface (getFiles / readFile). The
// archive's directory is parsed once into a name -> record map: the trailer
// (signature 0x06054b50, the last 22 bytes: no archive comment) gives the
// directory's extent and record count; each directory record (0x02014b50, 46
// fixed bytes + name + extra + comment) gives a member's compression method,
// stored size and local-record offset; a member's bytes follow its local
// record (0x04034b50, 30 fixed bytes + name + extra). Stored members (method 0,
// how BVP archives are written) are returned as they lie; deflated ones
// (method 8) are inflated with Node's zlib, which the reference does not do.
const ZIP_TRAILER = 0x06054b50, ZIP_DIRREC = 0x02014b50, ZIP_LOCAL = 0x04034b50;

class ZIPReader {
  constructor(loader) {
    this._loader = loader;
    this._members = null;  // Map: member name -> { method, stored, local }
  }

  async getFiles() {
    return Array.from((await this._directory()).keys());
  }

  async readFile(fileName) {
    const m = (await this._directory()).get(fileName);
    if (!m) throw new Error(`ZIPReader: the archive has no member named '${fileName}'`);
    const local = bytesView(await this._loader.readData(m.local, m.local + 30));
    if (local.getUint32(0, true) !== ZIP_LOCAL) {
      throw new Error(`ZIPReader: member '${fileName}' has no local record at byte ${m.local}`);
    }
    const first = m.local + 30 + local.getUint16(26, true) + local.getUint16(28, true);
    const raw = await this._loader.readData(first, first + m.stored);
    switch (m.method) {
      case 0: return raw;
      case 8: return new Uint8Array(zlib.inflateRawSync(Buffer.from(raw)));
      default: throw new Error(`ZIPReader: member '${fileName}' uses compression method ${m.method}`);
    }
  }

  async _directory() {
    if (this._members) return this._members;
    const total = await this._loader.readLength();
    const at = Math.max(total - 22, 0);
    const tail = bytesView(await this._loader.readData(at, total));
    if (tail.byteLength < 22 || tail.getUint32(0, true) !== ZIP_TRAILER) {
      throw new Error('ZIPReader: the last 22 bytes are not a zip trailer (archives with a comment are not read)');
    }
    const count = tail.getUint16(10, true), dirBytes = tail.getUint32(12, true), dirAt = tail.getUint32(16, true);
    const dir = await this._loader.readData(dirAt, dirAt + dirBytes);
    const v = bytesView(dir);
    const members = new Map();
    for (let k = 0, pos = 0; k < count; k++) {
      if (v.getUint32(pos, true) !== ZIP_DIRREC) throw new Error(`ZIPReader: directory record ${k} is damaged`);
      const nameLen = v.getUint16(pos + 28, true);
      const name = Buffer.from(dir.buffer, dir.byteOffset + pos + 46, nameLen).toString('utf8');
      members.set(name, { method: v.getUint16(pos + 10, true), stored: v.getUint32(pos + 20, true),
        local: v.getUint32(pos + 42, true) });
      pos += 46 + nameLen + v.getUint16(pos + 30, true) + v.getUint16(pos + 32, true);
    }
    this._members = members;
    return members;
  }
}

function bytesView(u8) {
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
