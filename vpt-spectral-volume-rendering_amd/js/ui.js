'use strict';
// Headless models of the three UI elements that produce the spectral renderer's
// inputs (SURVEY 8f f2). The reference's elements are DOM custom elements whose
// state is read by the renderer's 'change' handler (WebGPUMCMSpectralComputeRenderer.js:97-114);
// these classes keep the same state and the same derivations without a DOM, and
// emit the same 'change' events, so a Node host (or a test) can drive the HIP
// renderer exactly as the UI does:
//
//   MaterialTransferFunctionModel  ui/MaterialTransferFunction/MaterialTransferFunction.js
//     value: 256 x 256 rgba8 TF, texel (density row, wavelength column) =
//     (albedo, alpha, anisotropy, 0) of the material painted into that density row
//   SpectrumRepresentationModel    ui/SpectrumRepresentation/SpectrumRepresentation.js
//     n + 1 marker wavelengths on [400, 700] nm, placed by the exponential
//     spacing parameter k and rounded to whole nm as the markers display them
//   LightEditorModel               ui/LightEditor/LightEditor.js
//     256-entry spectral power distribution (default 100) and a direction
//
// Wiring: connectUiModels(renderer, {lightEditor, spectrumRepresentation,
// materialTransferFunction}) forwards each model's 'change' to the renderer's
// setter, like the reference's element listeners.

class Emitter {
  constructor() { this._listeners = new Map(); }
  addEventListener(type, fn) {
    if (!this._listeners.has(type)) this._listeners.set(type, []);
    this._listeners.get(type).push(fn);
  }
  removeEventListener(type, fn) {
    const l = this._listeners.get(type);
    if (l) this._listeners.set(type, l.filter(f => f !== fn));
  }
  dispatchEvent(ev) {
    for (const fn of this._listeners.get(ev.type) || []) fn(ev);
    return true;
  }
}

const TF_SIZE = 256;

class MaterialTransferFunctionModel extends Emitter {
  constructor() {
    super();
    this.materials = [];
    this.value = new Uint8Array(TF_SIZE * TF_SIZE * 4);  // all zero until painted
    this.selected_material_id = this.addMaterial().id;
  }

  // A new material: every wavelength entry 127 (the element's default).
  addMaterial(albedo, alpha, anisotropy) {
    const id = this.materials.reduce((m, x) => Math.max(m, x.id), 0) + 1;
    const arr = (a) => {
      const out = new Uint8Array(TF_SIZE).fill(127);
      if (a !== undefined) out.set(typeof a === 'number' ? new Uint8Array(TF_SIZE).fill(a) : a);
      return out;
    };
    const material = { id, albedo: arr(albedo), alpha: arr(alpha), anisotropy: arr(anisotropy) };
    this.materials.push(material);
    this.selected_material_id = id;
    return material;
  }

  // The last material cannot be removed; the first remaining one is selected.
  removeMaterial(id) {
    if (this.materials.length === 1) return false;
    const n = this.materials.length;
    this.materials = this.materials.filter(m => m.id !== id);
    if (this.materials.length === n) return false;
    this.selected_material_id = this.materials[0].id;
    return true;
  }

  // The editor's arrays for a material (albedo / alpha / anisotropy over 256 wavelengths).
  setMaterial(id, { albedo, alpha, anisotropy } = {}) {
    const m = this.materials.find(x => x.id === id);
    if (!m) throw new Error(`no material ${id}`);
    if (albedo) m.albedo = Uint8Array.from(albedo);
    if (alpha) m.alpha = Uint8Array.from(alpha);
    if (anisotropy) m.anisotropy = Uint8Array.from(anisotropy);
  }

  // Paint density rows [x0, x1] (either order, clamped to the canvas) with a
  // material, or clear them (erase: the ctrl-drag of the element).
  paint(x0, x1, id = this.selected_material_id, erase = false) {
    const m = this.materials.find(x => x.id === id);
    if (!m && !erase) throw new Error(`no material ${id}`);
    const lo = Math.max(0, Math.min(x0, x1)), hi = Math.min(TF_SIZE - 1, Math.max(x0, x1));
    for (let row = lo; row <= hi; row++) {
      for (let col = 0; col < TF_SIZE; col++) {
        const t = (row * TF_SIZE + col) * 4;
        this.value[t + 0] = erase ? 0 : m.albedo[col];
        this.value[t + 1] = erase ? 0 : m.alpha[col];
        this.value[t + 2] = erase ? 0 : m.anisotropy[col];
        this.value[t + 3] = 0;
      }
    }
    this.dispatchEvent({ type: 'change' });
  }
}

class SpectrumRepresentationModel extends Emitter {
  constructor(n_bins = 12, k = 0) {
    super();
    this.n_bins = n_bins;
    this.k = k;
    this.markers = [];  // positions on [0, 1] of the n + 1 markers
    this.arrange(k);
  }

  static toNm(x) { return 400 + x * 300; }

  // n + 1 markers at (e^{k t} - 1) / (e^k - 1), t = i / n (uniform for k = 0).
  arrange(k = this.k, n_bins = this.n_bins) {
    this.k = k;
    this.n_bins = n_bins;
    this.markers = [];
    for (let i = 0; i <= n_bins; i++) {
      const t = i / n_bins;
      this.markers.push(k === 0 ? t : (Math.exp(k * t) - 1) / (Math.exp(k) - 1));
    }
    this.dispatchEvent({ type: 'change' });
  }

  // Drag marker i to position x in [0, 1] (clamped, as the element clamps to its track).
  moveMarker(i, x) {
    this.markers[i] = Math.min(1, Math.max(0, x));
    this.dispatchEvent({ type: 'change' });
  }

  // The wavelengths the renderer reads: each marker's displayed whole-nm value, sorted.
  getBins() {
    return this.markers.map(x => Math.round(SpectrumRepresentationModel.toNm(x))).sort((a, b) => a - b);
  }
}

class LightEditorModel extends Emitter {
  constructor() {
    super();
    this.spectrum_power_distribution = new Uint8Array(256).fill(100);
    this.direction = [1, 0, 0];
  }
  setDirection(d) {
    this.direction = Array.from(d);
    this.dispatchEvent({ type: 'change' });
  }
  setSpectrum(spd) {
    if (spd.length !== 256) throw new Error('the light spectrum has 256 entries');
    this.spectrum_power_distribution = Uint8Array.from(spd);
    this.dispatchEvent({ type: 'change' });
  }
}

// Forward the models' changes to a renderer the way the reference's element
// listeners do (js:97-114): each change re-reads the model and resets.
function connectUiModels(renderer, { lightEditor, spectrumRepresentation, materialTransferFunction } = {}) {
  if (lightEditor) {
    const f = () => renderer.setLight(lightEditor.spectrum_power_distribution, lightEditor.direction);
    lightEditor.addEventListener('change', f);
    f();
  }
  if (spectrumRepresentation) {
    const f = () => renderer.setSpectrumRepresentation(spectrumRepresentation.getBins());
    spectrumRepresentation.addEventListener('change', f);
    f();
  }
  if (materialTransferFunction) {
    const f = () => renderer.setMaterialTransferFunction(materialTransferFunction.value);
    materialTransferFunction.addEventListener('change', f);
    f();
  }
}

module.exports = { MaterialTransferFunctionModel, SpectrumRepresentationModel, LightEditorModel,
  connectUiModels };
