'use strict';
// MCMComputeRenderer — drop-in for the reference's RGB sibling renderer
// WebGPUMCMComputeRenderer (src/js/renderers/WebGPUMCMComputeRenderer.js,
// shader src/wgsl/renderers/MCMComputeRenderer.wgsl; factory name
// 'mcm-compute', WebGPURendererFactory.js:21), running the RGB march on an
// MI355X (HIP k_march_rgb / k_reset_rgb behind the same C-ABI, renderer kind
// VPTMCM_RENDERER_RGB).
//
// Same constructor, properties (extinction, anisotropy, bounces, steps,
// transferFunction; js:19-59), 'change' -> reset semantics (js:61-77) and the
// base surface (render, reset, setVolume, setResolution, setTransferFunction,
// getTexture, destroy). The transfer function is an rgba8 image
// ({width, height, data}) as the reference's ImageBitmap/canvas; the environment
// is the rendering context's 1x1 texel ({width: 1, height: 1, data}).
const { PropertyBag } = require('./PropertyBag');
const { mvpInverse } = require('./Camera');
const { native, f32bits } = require('./MCMSpectralComputeRenderer');

const LAYOUTS = { linear: 0, corner8: 1, brick8: 2, column4: 3 };
const RENDERER_RGB = 1;
const RESET_ON = ['extinction', 'anisotropy', 'bounces', 'transferFunction'];  // js:70-75

function imageOf(tf) {
  if (tf && tf.data && tf.width && tf.height) return tf;
  if (tf instanceof Uint8Array || tf instanceof Uint8ClampedArray) {
    return { width: tf.length / 4, height: 1, data: tf };  // one row of rgba8 texels
  }
  throw new Error('transfer function must be an rgba8 image {width, height, data}');
}

class MCMComputeRenderer extends PropertyBag {
  constructor(device, volume, camera, environment, options = {}) {
    super();
    this._resolution = options.resolution !== undefined ? options.resolution : 512;
    this._workgroup_size = options.workgroup_size || [8, 8];
    this._device = typeof device === 'number' ? { ordinal: device } : (device || {});
    this._volume = volume || null;
    this._camera = camera;
    this._environment = environment || null;
    this._random = options.random || Math.random;

    this.registerProperties([  // js:19-59
      { name: 'extinction', label: 'Extinction', type: 'spinner', value: 1, min: 0 },
      { name: 'anisotropy', label: 'Anisotropy', type: 'slider', value: 0, min: -1, max: 1 },
      { name: 'bounces', label: 'Max bounces', type: 'spinner', value: 8, min: 0 },
      { name: 'steps', label: 'Steps', type: 'spinner', value: 8, min: 0 },
      { name: 'transferFunction', label: 'Transfer function', type: 'transfer-function',
        value: new Uint8Array(256) },
    ]);
    this.addEventListener('change', e => {  // js:61-77
      const { name } = e.detail || {};
      if (name === 'transferFunction') this.setTransferFunction(this.transferFunction);
      if (RESET_ON.includes(name)) this.reset();
    });
    this._createNative();
  }

  _createNative() {
    const layout = LAYOUTS[this._device.layout || 'column4'];
    if (layout === undefined) throw new Error(`unknown volume layout '${this._device.layout}'`);
    const ordinal = this._device.ordinal !== undefined ? this._device.ordinal : -1;
    this._h = native().create(this._resolution, ordinal, layout, RENDERER_RGB);
    if (this._tfImage) this._uploadTF(this._tfImage);  // else the ctor's 2x1 default (base :23-28)
    if (this._environment && this._environment.data) {
      const e = this._environment;
      native().setEnvironment(this._h, Uint8Array.from(e.data), e.width || 1, e.height || 1);
    }
    this._volumeReady = false;
    if (this._volume) this._uploadVolume(this._volume);
  }

  // ---- the plugin surface (WebGPUAbstractComputeRenderer.js:41-85) ----
  render() {
    if (!this._volumeReady) throw new Error('render: no volume loaded (setVolume first)');
    const m = mvpInverse(this._camera);
    native().setParams(this._h, this.extinction, this.anisotropy, this.bounces, this.steps, 0);  // js:186-197
    native().render(this._h, m, f32bits(this._random()));
  }

  reset() {
    native().reset(this._h, mvpInverse(this._camera), f32bits(this._random()));
  }

  setVolume(volume) {
    this._volume = volume;
    this._uploadVolume(volume);
    this.reset();
  }

  async loadVolume(volume) {  // block-wise HBM ingest (readModality's placements), then reset
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

  setTransferFunction(transferFunction) {  // base :62-69 (rgba8unorm-srgb texture)
    this._tfImage = imageOf(transferFunction);
    this._uploadTF(this._tfImage);
  }

  setResolution(resolution) {
    if (resolution !== this._resolution) {
      this._resolution = resolution;
      native().destroy(this._h);
      this._createNative();
      this.reset();
    }
  }

  getTexture() {
    const R = this._resolution;
    const data = new Uint16Array(R * R * 4);
    native().readRGBA16F(this._h, data, R);
    return { width: R, height: R, format: 'rgba16float', data };
  }

  // The last pass's fp32 radiance (before the rgba16float store): parity checks.
  getRadianceRGB() {
    const R = this._resolution;
    const data = new Float32Array(R * R * 3);
    native().readRGB(this._h, data, R);
    return { width: R, height: R, format: 'rgb32float', data };
  }

  getTextureSampler() {
    return { addressModeU: 'clamp-to-edge', addressModeV: 'clamp-to-edge', magFilter: 'nearest',
      minFilter: 'nearest' };
  }

  destroy() {
    if (this._h) native().destroy(this._h);
    this._h = null;
  }

  // ---- extensions ----
  // n render() calls in one enqueue (fused into 32-pass launches)
  renderPasses(n) {
    if (!this._volumeReady) throw new Error('render: no volume loaded (setVolume first)');
    const m = mvpInverse(this._camera);
    native().setParams(this._h, this.extinction, this.anisotropy, this.bounces, this.steps, 0);
    const seeds = new Uint32Array(n);
    for (let k = 0; k < n; k++) seeds[k] = f32bits(this._random());
    native().renderPasses(this._h, m, seeds);
  }

  // What the last march launch ran: { mode, tpl, spec, passes, launches }
  lastLaunch() {
    return native().lastLaunch(this._h);
  }

  readPhotons() {  // 64-B Photon records (Photon.wgsl)
    const R = this._resolution;
    const out = new Uint8Array(R * R * 64);
    native().readPhotons(this._h, out, R);
    return out;
  }

  synchronize() {
    native().synchronize(this._h);
  }

  _uploadTF(img) {
    native().setTransferFunction(this._h, Uint8Array.from(img.data), img.width, img.height);
  }

  _uploadVolume(volume) {
    const v = volume && (volume.data ? volume : volume.hostVolume);
    if (!v || !v.data) {
      this._volumeReady = false;
      return;
    }
    native().setVolume(this._h, v.data, v.width, v.height, v.depth);
    this._volumeReady = true;
  }
}

module.exports = { MCMComputeRenderer };
