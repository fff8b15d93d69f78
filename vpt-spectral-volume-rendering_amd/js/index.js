'use strict';
// Public JS surface of the MI355X spectral MCM renderer.
const { MCMSpectralComputeRenderer, native } = require('./MCMSpectralComputeRenderer');
const { RendererFactory } = require('./RendererFactory');
const { MCMComputeRenderer } = require('./MCMComputeRenderer');
const { ArtisticToneMapper, ToneMapperFactory } = require('./ArtisticToneMapper');
const { Camera, Transform, PerspectiveCamera, mvpInverse } = require('./Camera');
const { PropertyBag } = require('./PropertyBag');
const { BufferLoader, FileLoader, RAWReader, ZIPReader, BVPReader, ReaderFactory, Volume } = require('./readers');
const spectrum = require('./spectrum');
const ui = require('./ui');
const mat4 = require('./mat4');

// A HIP device descriptor in place of the reference's GPUDevice: one ordinal,
// or a list of ordinals for one renderer driving several GPUs (a
// photon-parallel replica per GPU, composited on the first; transport 'peer'
// or 'rccl', include/vptmcm.h).
function createDevice(ordinal = 0, layout = 'column4', transport = 'peer') {
  if (Array.isArray(ordinal)) return { devices: ordinal.slice(), layout, transport };
  return { ordinal, layout };
}

module.exports = {
  MCMSpectralComputeRenderer, MCMComputeRenderer, RendererFactory, ArtisticToneMapper, ToneMapperFactory, Camera, Transform, PerspectiveCamera, mvpInverse,
  PropertyBag, BufferLoader, FileLoader, RAWReader, ZIPReader, BVPReader, ReaderFactory, Volume, spectrum, mat4, createDevice, native,
  ui, MaterialTransferFunctionModel: ui.MaterialTransferFunctionModel,
  SpectrumRepresentationModel: ui.SpectrumRepresentationModel, LightEditorModel: ui.LightEditorModel,
  connectUiModels: ui.connectUiModels,
};
