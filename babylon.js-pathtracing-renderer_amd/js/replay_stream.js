// replay_stream.js — replays a recorded per-frame draw stream (tests/golden/*.json: the uniforms,
// sampler bindings and draw order a reference setup script issued) through the Babylon-shaped
// shim and the N-API addon on an MI355X, then writes the accumulation texture and the canvas.
// This is the JavaScript host path on machines that have the GPU but not the reference scripts.
//
// usage: node replay_stream.js <stream.json> <payload_dir> <out_prefix> [frames]
//   (PT_DEVICES="0,0" etc. renders through a multi-part context: the frame split over the parts)
//   payload_dir holds bluenoise.u8 (256x256 RGBA8) and, for glTF streams, bvh.f32 / tri.f32
//   (2048x2048 RGBA32F, the RawTexture payloads), hdr.f32 for HDRI streams (the environment), and
//   optionally maps.json (model PBR maps, below).
'use strict';
const fs = require('fs');
const path = require('path');
const { install } = require('./babylon_pt.js');

const [streamPath, payloadDir, outPrefix, framesArg] = process.argv.slice(2);
const meta = JSON.parse(fs.readFileSync(streamPath, 'utf8'));
const nFrames = framesArg ? parseInt(framesArg, 10) : meta.frames.length;
const BABYLON = {};
const errors = [];
install(BABYLON, { width: meta.width, height: meta.height, onError: (m) => errors.push(m) });
const PROGRAMS = { cornell: 3, gltf: 4, hdri: 5, sky: 6, quadric: 7, skymesh: 8 };
const SHADER_PROGRAM = { screenCopyFragmentShader: 1, screenOutputFragmentShader: 2 };

const engine = new BABYLON.Engine({ width: meta.width, height: meta.height });
const f32 = (f) => { const b = fs.readFileSync(path.join(payloadDir, f)); return new Float32Array(b.buffer, b.byteOffset, b.byteLength / 4); };
const tex = {
  pathTracingRenderTarget: new BABYLON.RenderTargetTexture('pathTracingRenderTarget', { width: meta.width, height: meta.height }, engine),
  screenCopyRenderTarget: new BABYLON.RenderTargetTexture('screenCopyRenderTarget', { width: meta.width, height: meta.height }, engine),
  'file:BlueNoise_RGBA256.png': BABYLON.RawTexture.CreateRGBATexture(new Uint8Array(fs.readFileSync(path.join(payloadDir, 'bluenoise.u8'))), 256, 256, engine, false, false, 1, 0),
};
if (meta.textures) {
  for (const [raw, kind] of Object.entries(meta.textures)) {
    // the HDRI scene's environment: its own size, invertY and trilinear sampling, as the script uploads it
    tex[raw] = kind === 'hdr'
      ? BABYLON.RawTexture.CreateRGBATexture(f32('hdr.f32'), meta.hdr.width, meta.hdr.height, engine, false, meta.hdr.invertY, 3, 1)
      : BABYLON.RawTexture.CreateRGBATexture(f32(kind + '.f32'), 2048, 2048, engine, false, false, 1, 1);
  }
}
// maps.json (optional): { texture name: image file } - model maps as Babylon's glTF loader leaves
// them (a texture holding the image file's bytes, invertY false); the shim decodes and uploads them
// when the script binds them (setTexture)
const mapsSpec = path.join(payloadDir, 'maps.json');
if (fs.existsSync(mapsSpec)) {
  for (const [name, file] of Object.entries(JSON.parse(fs.readFileSync(mapsSpec, 'utf8')))) {
    tex[name] = { name, url: 'data:' + file, _buffer: new Uint8Array(fs.readFileSync(file)), samplingMode: 3, _invertY: false };
  }
}
const renderer = new BABYLON.EffectRenderer(engine);
const wrappers = {};
for (const call of meta.frames[0]) {
  wrappers[call.effect] = new BABYLON.EffectWrapper({ engine, name: call.effect, uniformNames: Object.keys(call.uniforms),
    samplerNames: Object.keys(call.samplers), ptProgram: SHADER_PROGRAM[call.shader] || PROGRAMS[meta.scene] });
}
for (let i = 0; i < nFrames; i++) {
  for (const call of meta.frames[i]) {
    const w = wrappers[call.effect];
    w.onApplyObservable.clear();
    w.onApplyObservable.add(() => {
      for (const [n, [kind, v]] of Object.entries(call.uniforms)) {
        if (kind === 'i') w.effect.setInt(n, v[0]);
        else if (v.length === 16) w.effect.setMatrix(n, { m: v });
        else if (v.length === 1) w.effect.setFloat(n, v[0]);
        else if (v.length === 2) w.effect.setFloat2(n, v[0], v[1]);
        else w.effect.setFloat3(n, v[0], v[1], v[2]);
      }
      for (const [n, t] of Object.entries(call.samplers)) w.effect.setTexture(n, t ? tex[t] : null);
    });
    renderer.render(w, call.target ? tex[call.target] : null);
  }
}
fs.writeFileSync(outPrefix + '.acc.f32', Buffer.from(tex.pathTracingRenderTarget.readPixels().buffer));
fs.writeFileSync(outPrefix + '.canvas.u8', Buffer.from(engine.readCanvas().buffer));
if (errors.length) { console.error(errors.join('\n')); process.exit(2); }
engine.dispose();
