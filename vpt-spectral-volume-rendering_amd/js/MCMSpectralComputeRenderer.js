'use strict';
// MCMSpectralComputeRenderer — drop-in replacement for the reference's
// WebGPUMCMSpectralComputeRenderer (src/js/renderers/WebGPUMCMSpectralComputeRenderer.js)
// and its base WebGPUAbstractComputeRenderer, running the march on an MI355X
// through the N-API shim (napi/vptmcm_napi.c) and the C-ABI (include/vptmcm.h).
//
// Same constructor signature, properties, 'change' semantics and methods:
//   render()            -> _renderFrame (js:262-376): uploads light/TF/uniforms/
//                          spectrum, one march pass with a fresh Math.random() seed
//   reset()             -> _resetFrame (js:213-260): full photon re-initialisation
//   setVolume(volume)   -> base :57-60 (+ reset)
//   setResolution(n)    -> base :71-77 (+ reset)
//   setTransferFunction -> base :62-69 (kept for the surface; unused by the kernel)
//   getTexture()        -> the rgba16float radiance image (host copy: a HIP
//                          renderer cannot hand out a GPUTexture); with a
//                          device list, the composite of every GPU's photons
//   destroy()           -> js:207-211
// DOM reads of the reference (#light-editor, #spectrum-representation,
// #material-transfer-function) become explicit setters and change-event payloads.
const path = require('path');
const { PropertyBag } = require('./PropertyBag');
const { mvpInverse } = require('./Camera');
const spectrum = require('./spectrum');

let addon = null;
function native() {
  if (!addon) {
    const p = path.join(__dirname, '..', 'lib', 'vptmcm_napi.node');
    try {
      addon = require(p);
    } catch (e) {
      throw new Error(`HIP renderer addon not available at ${p} (build with ` +
        `\`python __graft_entry__.py build\`): ${e.message}`);
    }
  }
  return addon;
}

const LAYOUTS = { linear: 0, corner8: 1, brick8: 2, column4: 3 };
const TRANSPORTS = { peer: 0, rccl: 1 };  // vptmcm_config::group_transport
const RESET_ON = ['extinction', 'anisotropy', 'bounces', 'materialTransferFunction',
  'spectrumRepresentation', 'lightEditor'];  // js:116-125

function f32bits(x) {
  const f = new Float32Array([x]);
  return new Uint32Array(f.buffer)[0];
}

class MCMSpectralComputeRenderer extends PropertyBag {
  // device: { ordinal, layout } (or a device ordinal), or { devices: [ordinals],
  // layout, transport } for one renderer driving several GPUs (one
  // photon-parallel replica per entry; options.devices works too; transport
  // 'peer' (default, deterministic ordered composite) or 'rccl'); volume: a Volume (readers.js)
  // or an object with { data, width, height, depth }; camera: Camera.js or the
  // reference's camera node; environment: accepted and ignored, as the kernel's
  // environment sampling is dead code (wgsl:144-146).
  constructor(device, volume, camera, environment, options = {}) {
    super();
    this._resolution = options.resolution !== undefined ? options.resolution : 512;
    this._workgroup_size = options.workgroup_size || [8, 8];
    this._device = typeof device === 'number' ? { ordinal: device } : Object.assign({}, device || {});
    if (options.devices && !this._device.devices) this._device.devices = options.devices;
    this._volume = volume || null;
    this._camera = camera;
    this._environment = environment;
    this._random = options.random || Math.random;
    this._cie = options.cie || null;

    this.registerProperties([  // js:19-73
      { name: 'extinction', label: 'Extinction', type: 'spinner', value: 1, min: 0 },
      { name: 'anisotropy', label: 'Anisotropy', type: 'slider', value: 0, min: -1, max: 1 },
      { name: 'bounces', label: 'Max bounces', type: 'spinner', value: 8, min: 0 },
      { name: 'steps', label: 'Steps', type: 'spinner', value: 8, min: 0 },
      { name: 'spectrumRepresentation', label: 'Spectrum representation',
        type: 'spectrum-representation', id: 'spectrum-representation' },
      { name: 'lightEditor', label: 'Light editor', type: 'light-editor', id: 'light-editor' },
      { name: 'materialTransferFunction', label: 'Material transfer function',
        type: 'material-transfer-function', id: 'material-transfer-function' },
    ]);

    this.max_n_bins = 12;  // js:76, MAX_N_BINS
    this.n_bins = 12;
    this.spectrumRepresentationData = spectrum.DEFAULT_BINS.slice();
    this._spectrumBuffer = options.spectrumBuffer ? Float32Array.from(options.spectrumBuffer) : null;
    if (!this._spectrumBuffer) this.compute_spectral_coefficients();

    this.light_direction = [1, 0, 0];  // js:82-83
    this.light_spectrum_power_distribution = new Uint8Array(256).fill(100);
    this.material_transfer_function = new Uint8Array(256 * 256 * 4);

    this.addEventListener('change', e => this._onChange(e.detail || {}));  // js:89-126

    this._createNative();
  }

  _createNative() {
    const layout = LAYOUTS[this._device.layout || 'column4'];
    if (layout === undefined) throw new Error(`unknown volume layout '${this._device.layout}'`);
    const ordinal = this._device.ordinal !== undefined ? this._device.ordinal : -1;
    const devs = this._device.devices;
    if (devs !== undefined) {
      if (!Array.isArray(devs) || devs.length < 1 || devs.length > 8)
        throw new Error('devices: an array of 1 to 8 device ordinals');
      const transport = TRANSPORTS[this._device.transport || 'peer'];
      if (transport === undefined) throw new Error(`unknown transport '${this._device.transport}'`);
      this._h = native().create(this._resolution, ordinal, layout, 0, devs.map(d => d | 0), transport);
    } else {
      this._h = native().create(this._resolution, ordinal, layout);
    }
    this._dirty = { light: true, tf: true, spectrum: true };
    this._volumeReady = false;
    if (this._volume) this._uploadVolume(this._volume);
  }

  _onChange({ name, value }) {
    if (name === 'transferFunction') this.setTransferFunction(this.transferFunction);
    if (name === 'lightEditor' && value) {
      if (value.spectrum_power_distribution) this.setLight(value.spectrum_power_distribution,
        value.direction || this.light_direction, false);
    }
    if (name === 'spectrumRepresentation' && value) this.setSpectrumRepresentation(value, false);
    if (name === 'materialTransferFunction' && value) this.setMaterialTransferFunction(value, false);
    if (RESET_ON.includes(name)) this.reset();
  }

  // ---- DOM-free inputs (the reference reads these from UI elements) ----
  setLight(spd, direction, announce = true) {
    if (spd.length !== 256) throw new Error('light SPD must have 256 entries');
    this.light_spectrum_power_distribution = Uint8Array.from(spd);
    this.light_direction = Array.from(direction);
    this._dirty.light = true;
    if (announce) this.dispatchEvent({ type: 'change', detail: { name: 'lightEditor' } });
  }

  setSpectrumRepresentation(bins, announce = true) {
    if (bins.length - 1 > this.max_n_bins) throw new Error('at most 12 spectral bins');
    this.spectrumRepresentationData = Array.from(bins);
    this.n_bins = bins.length - 1;
    this._spectrumBuffer = null;
    this.compute_spectral_coefficients();
    if (announce) this.dispatchEvent({ type: 'change', detail: { name: 'spectrumRepresentation' } });
  }

  setMaterialTransferFunction(rgba, announce = true) {
    if (rgba.length !== 256 * 256 * 4) throw new Error('material TF must be 256x256 RGBA8');
    this.material_transfer_function = Uint8Array.from(rgba);
    this._dirty.tf = true;
    if (announce) this.dispatchEvent({ type: 'change', detail: { name: 'materialTransferFunction' } });
  }

  // js:379-412 (needs the host application's CIE table, options.cie)
  compute_spectral_coefficients() {
    if (!this._cie) {
      throw new Error('compute_spectral_coefficients needs the CIE table (options.cie, ' +
        'e.g. CIE_SPECTRUM from the application\'s utils/Spectrum.js) or options.spectrumBuffer');
    }
    const c = spectrum.computeSpectralCoefficients(this.spectrumRepresentationData, this._cie);
    this.x_coeff = c.x;
    this.y_coeff = c.y;
    this.z_coeff = c.z;
    this._dirty && (this._dirty.spectrum = true);
  }

  spectrumBuffer() {
    if (this._spectrumBuffer) return this._spectrumBuffer;
    return spectrum.packSpectrumBuffer(this.spectrumRepresentationData,
      { x: this.x_coeff, y: this.y_coeff, z: this.z_coeff });
  }

  // ---- the plugin surface (WebGPUAbstractComputeRenderer.js:41-85) ----
  render() {
    this._renderFrame();
  }

  reset() {
    this._resetFrame();
  }

  setVolume(volume) {
    this._volume = volume;
    this._uploadVolume(volume);
    this.reset();
  }

  // Streams the volume's blocks straight into HBM (readModality's per-placement
  // writes, WebGPUVolume.js:67-93), then resets; for large (bricked) volumes.
  async loadVolume(volume) {
    const A = native();
    const h = this._h;
    await volume.load({
      begin: (w, hh, d) => A.volumeBegin(h, w, hh, d),
      block: (data, x, y, z, w, hh, d) => A.volumeWriteBlock(h, data, x, y, z, w, hh, d),
      end: () => A.volumeEnd(h),
    });
    this._volume = volume;
    this._volumeReady = true;
    this.reset();
  }

  setTransferFunction(transferFunction) {
    this._transferFunction = transferFunction;  // base :62-69; not read by the spectral kernel
  }

  setResolution(resolution) {
    if (resolution !== this._resolution) {
      this._resolution = resolution;
      native().destroy(this._h);
      this._createNative();  // photons are re-allocated for the new R (see DESIGN.md)
      this.reset();
    }
  }

  getTexture() {
    const R = this._resolution;
    const data = new Uint16Array(R * R * 4);
    native().readRGBA16F(this._h, data, R);
    return { width: R, height: R, format: 'rgba16float', data };
  }

  // The last pass's fp32 RGB (radiance_to_rgb before the rgba16float store,
  // wgsl:304-326): not part of the reference surface, used for fp32 parity checks.
  getRadianceRGB() {
    const R = this._resolution;
    const data = new Float32Array(R * R * 3);
    native().readRGB(this._h, data, R);
    return { width: R, height: R, format: 'rgb32float', data };
  }

  getTextureSampler() {
    return { addressModeU: 'clamp-to-edge', addressModeV: 'clamp-to-edge', magFilter: 'nearest',
      minFilter: 'nearest' };  // base :102-107
  }

  destroy() {
    if (this._h) native().destroy(this._h);
    this._h = null;
  }

  // ---- extensions beyond the reference surface ----
  // n render() calls in one enqueue: the same uploads, then n passes with n
  // fresh seeds (launched as fused multi-pass marches, 32 passes per launch)
  renderPasses(n) {
    if (!this._volumeReady) throw new Error('render: no volume loaded (setVolume first)');
    const m = this._matrix();
    this._uploadTables();
    const seeds = new Uint32Array(n);
    for (let k = 0; k < n; k++) seeds[k] = this._seedBits();
    native().renderPasses(this._h, m, seeds);
  }

  // The GPUs this renderer drives (its device list; one entry without one).
  devices() {
    return native().groupDevices(this._h);
  }

  // Enqueue the composite of the current frame over the GPUs (asynchronous;
  // getTexture() makes it when it is missing). A progressive display calls it
  // once per shown frame, right after that frame's render().
  composite() {
    native().composite(this._h);
  }

  // What the last march launch ran: { mode, tpl, spec, passes, launches }
  // (vptmcm_debug_last_launch; launches counts every march launch so far)
  lastLaunch() {
    return native().lastLaunch(this._h);
  }

  // Mode B (DESIGN.md): march only pixel rows [y0, y1) (multiples of 8; y1 may
  // be the resolution); ranks holding disjoint bands composite with
  // native().commGatherBands. A new resolution drops the band.
  setBand(y0, y1) {
    native().setBand(this._h, y0, y1);
  }

  readPhotons() {
    const R = this._resolution;
    const out = new Uint8Array(R * R * 144);
    native().readPhotons(this._h, out, R);
    return out;
  }

  synchronize() {
    native().synchronize(this._h);
  }

  // ---- internals ----
  _uploadVolume(volume) {
    const v = volume && (volume.data ? volume : volume.hostVolume);
    if (!v || !v.data) {
      this._volumeReady = false;  // like getTexture() === null before load (WebGPUVolume.js:127-132)
      return;
    }
    native().setVolume(this._h, v.data, v.width, v.height, v.depth);
    this._volumeReady = true;
  }

  _matrix() {
    return mvpInverse(this._camera);
  }

  _seedBits() {
    return f32bits(this._random());  // Float32Array([Math.random()]) -> bitcast (js:298, wgsl:122)
  }

  _uploadTables() {
    const A = native();
    if (this._dirty.light) {
      A.setLight(this._h, this.light_spectrum_power_distribution, Float32Array.from(this.light_direction));
      this._dirty.light = false;
    }
    if (this._dirty.tf) {
      A.setMaterialTF(this._h, this.material_transfer_function);
      this._dirty.tf = false;
    }
    // rewritten every pass like the reference's UBO (js:295-309); the library
    // ignores unchanged values, so queued render() passes stay fused
    A.setParams(this._h, this.extinction, this.anisotropy, this.bounces, this.steps, 0);  // blur 0, js:299
    if (this._dirty.spectrum) {
      A.setSpectrum(this._h, this.spectrumBuffer());  // only in _renderFrame (js:311-312)
      this._dirty.spectrum = false;
    }
  }

  _resetFrame() {
    native().reset(this._h, this._matrix(), this._seedBits());
  }

  _renderFrame() {
    if (!this._volumeReady) {
      // the reference fails here too: this._volume.getTexture() is null (js:320)
      throw new Error('render: no volume loaded (setVolume first)');
    }
    const m = this._matrix();
    this._uploadTables();
    native().render(this._h, m, this._seedBits());
  }
}

module.exports = { MCMSpectralComputeRenderer, native, f32bits };
