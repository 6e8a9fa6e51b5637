// babylon_pt.js — the drop-in: Babylon's effect API (EffectWrapper / EffectRenderer /
// RenderTargetTexture / RawTexture / Texture / Engine render loop) implemented over libpt.so through
// the N-API addon, so the reference's unmodified js/*_Path_Tracing.js setup scripts render on an
// MI355X. Everything else those scripts use (Vector3, Matrix, TransformNode, UniversalCamera,
// SceneLoader, Mesh.MergeMeshes, the glTF loader) stays the real Babylon running on NullEngine:
// the scene graph is host-side bookkeeping, the pixels are produced by the gfx950 kernels.
//
//   const BABYLON = require('babylonjs');              // the vendored build the page loads
//   require('.../js/babylon_pt.js').install(BABYLON, { width: 1920, height: 1080 });
//   // ...then load js/PathTracingCommon.js, the scene shader and the setup script unchanged.
//
// Boundary map (reference call -> C ABI, include/pt.h):
//   new BABYLON.Engine(canvas)                    -> pt_ctx_create           (js/GLTF_Model_Path_Tracing.js:189)
//   new BABYLON.RenderTargetTexture(n,{w,h},...)  -> pt_render_target_create (:762-768), .resize -> pt_render_target_resize
//   BABYLON.RawTexture.CreateRGBATexture(...)     -> pt_texture_create_rgba32f / _rgba8 (:466-487)
//   new BABYLON.Texture(url, ...)                 -> host PNG / JPEG decode + pt_texture_create_rgba8 (:749-758);
//   Texture.updateURL(url, bytes) (glTF loader)   -> the same, for the models' PBR maps
//                                                    '*.hdr' -> host RGBE decode, readPixels() (js/HDRI_Environment_Path_Tracing.js:764-823)
//   new BABYLON.EffectWrapper({...})              -> pt_effect_create (GLSL text -> program) (:773-811)
//   effect.setFloat/.../setMatrix/setTexture      -> pt_set_float / pt_set_int / pt_set_texture (:813-848)
//   new BABYLON.EffectRenderer(engine).render()   -> pt_render (:1230-1235)
'use strict';
const fs = require('fs');
const path = require('path');
const zlib = require('zlib');

const ERR = { 0: 'PT_OK', '-1': 'PT_ERR_ARG', '-2': 'PT_ERR_HIP', '-3': 'PT_ERR_SHADER', '-4': 'PT_ERR_STATE',
  '-5': 'PT_ERR_OOM', '-6': 'PT_ERR_DEVICE', '-7': 'PT_ERR_UNSUPPORTED', '-8': 'PT_ERR_DATA' };
const TEXTURETYPE_UNSIGNED_BYTE = 0;

function loadAddon() {
  return require(path.join(__dirname, '..', 'napi', 'pt_napi.node'));
}

// ---------------------------------------------------------------------------------- Radiance .hdr
// The HDRI scene loads its environment with new BABYLON.Texture('*.hdr', ..., onLoad) and reads it
// back with readPixels() (js/HDRI_Environment_Path_Tracing.js:764-823). RGBE -> float as Babylon's
// HDRTools: value = mantissa * 2^(exponent - 136), exponent 0 -> 0; scanlines in file order (the
// usual "-Y H +X W" orientation: first scanline = top row = first row of the returned data), alpha 1.
// Both the flat layout and the adaptive run-length scanlines (2,2,hi,lo header) are read.
function decodeHDR(buf) {
  let pos = 0;
  const line = () => { const e = buf.indexOf(10, pos); const l = buf.toString('latin1', pos, e); pos = e + 1; return l; };
  const magic = line();
  if (!magic.startsWith('#?')) throw new Error('not a Radiance HDR file');
  let fmt = '';
  for (let l = line(); l !== ''; l = line()) if (l.startsWith('FORMAT=')) fmt = l.slice(7);
  if (fmt && fmt !== '32-bit_rle_rgbe') throw new Error('unsupported HDR format ' + fmt);
  const m = /^-Y (\d+) \+X (\d+)$/.exec(line().trim());
  if (!m) throw new Error('unsupported HDR orientation');
  const h = parseInt(m[1], 10), w = parseInt(m[2], 10);
  const data = new Float32Array(w * h * 4);
  const rgbe = new Uint8Array(w * 4);
  for (let y = 0; y < h; y++) {
    if (w >= 8 && w < 0x8000 && buf[pos] === 2 && buf[pos + 1] === 2 && ((buf[pos + 2] << 8) | buf[pos + 3]) === w) {
      pos += 4;
      for (let c = 0; c < 4; c++) {
        for (let x = 0; x < w;) {
          let n = buf[pos++];
          if (n > 128) { n -= 128; const v = buf[pos++]; for (let k = 0; k < n; k++) rgbe[4 * (x++) + c] = v; }
          else for (let k = 0; k < n; k++) rgbe[4 * (x++) + c] = buf[pos++];
        }
      }
    } else {
      for (let x = 0; x < 4 * w; x++) rgbe[x] = buf[pos++];
    }
    for (let x = 0; x < w; x++) {
      const e = rgbe[4 * x + 3], o = 4 * (y * w + x);
      const f = e ? Math.pow(2, e - 136) : 0;
      data[o] = rgbe[4 * x] * f; data[o + 1] = rgbe[4 * x + 1] * f; data[o + 2] = rgbe[4 * x + 2] * f; data[o + 3] = 1;
    }
  }
  return { width: w, height: h, data };
}

// ---------------------------------------------------------------------------------- PNG (RGBA8/16)
// The blue-noise texture is a 16-bit RGBA PNG; WebGL samples it as 8-bit. Pinned: high byte.
function decodePNG(buf) {
  if (buf.readUInt32BE(0) !== 0x89504e47) throw new Error('not a PNG');
  let pos = 8, w = 0, h = 0, bd = 0, ct = 0;
  const idat = [];
  while (pos < buf.length) {
    const len = buf.readUInt32BE(pos), type = buf.toString('ascii', pos + 4, pos + 8);
    const body = buf.slice(pos + 8, pos + 8 + len);
    if (type === 'IHDR') { w = body.readUInt32BE(0); h = body.readUInt32BE(4); bd = body[8]; ct = body[9]; if (body[12]) throw new Error('interlaced PNG'); }
    else if (type === 'IDAT') idat.push(body);
    pos += 12 + len;
  }
  const ch = { 6: 4, 2: 3, 0: 1, 4: 2 }[ct];
  if (!ch || (bd !== 8 && bd !== 16)) throw new Error('unsupported PNG format');
  const bpp = ch * bd / 8, stride = w * bpp;
  const raw = zlib.inflateSync(Buffer.concat(idat));
  const cur = Buffer.alloc(stride), prev = Buffer.alloc(stride);
  const out = new Uint8Array(w * h * 4);
  for (let y = 0, p = 0; y < h; y++) {
    const ft = raw[p++];
    for (let x = 0; x < stride; x++) {
      const a = x >= bpp ? cur[x - bpp] : 0, b = prev[x], c = x >= bpp ? prev[x - bpp] : 0;
      let v = raw[p++];
      if (ft === 1) v += a; else if (ft === 2) v += b; else if (ft === 3) v += (a + b) >> 1;
      else if (ft === 4) { const pa = Math.abs(b - c), pb = Math.abs(a - c), pc = Math.abs(a + b - 2 * c); v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c); }
      cur[x] = v & 255;
    }
    for (let x = 0; x < w; x++) {
      const px = [0, 0, 0, 255];
      for (let k = 0; k < ch; k++) px[k] = cur[x * bpp + k * (bd / 8)];   // 16-bit: high byte
      if (ch === 1) { px[1] = px[2] = px[0]; }
      if (ch === 2) { px[3] = px[1]; px[1] = px[2] = px[0]; }
      out.set(px, 4 * (y * w + x));
    }
    cur.copy(prev);
  }
  return { width: w, height: h, data: out };
}

// ---------------------------------------------------------------------------------- JPEG (host)
// JPEG maps (the glTF models' PBR textures) are decoded by libpt (pt_jpeg_decode_rgba8,
// csrc/pt_jpeg.cpp: libjpeg-turbo's default decompression reproduced bit for bit), through the addon.
function decodeImage(buf, addon) {
  buf = Buffer.from(buf.buffer ? Buffer.from(buf.buffer, buf.byteOffset, buf.byteLength) : buf);
  if (buf.length >= 4 && buf.readUInt32BE(0) === 0x89504e47) return decodePNG(buf);
  if (!(buf.length >= 2 && buf[0] === 0xff && buf[1] === 0xd8)) throw new Error('not a PNG or JPEG image');
  addon = addon || loadAddon();
  const wh = addon.pt_jpeg_size(buf);
  if (typeof wh === 'number') throw new Error('JPEG: ' + (ERR[wh] || wh));
  const data = new Uint8Array(4 * wh[0] * wh[1]);
  const rc = addon.pt_jpeg_decode_rgba8(buf, data);
  if (rc < 0) throw new Error('JPEG: ' + (ERR[rc] || rc));
  return { width: wh[0], height: wh[1], data };
}

function install(BABYLON, opts) {
  opts = Object.assign({ device: 0, width: 1920, height: 1080, baseDir: process.cwd(), addon: null, onError: null,
                        label: null }, opts || {});
  const addon = opts.addon || loadAddon();
  // opts.label(handle, name): optional debug hook naming each native handle (tracing tools)
  const label = (h, name) => { if (opts.label && h && typeof h !== 'number') opts.label(h, name); return h; };
  const report = opts.onError || ((msg) => console.error('[babylon_pt] ' + msg));
  // with the real Babylon loaded, the scene graph runs on its NullEngine; without it (e.g. a replay
  // host on the GPU box) a minimal base keeps the render-size bookkeeping
  const RealNull = BABYLON.NullEngine || class {
    constructor(o) { this._options = o; }
    getRenderWidth() { return this._options.renderWidth; }
    getRenderHeight() { return this._options.renderHeight; }
    dispose() {}
  };
  const set = (k, v) => { try { BABYLON[k] = v; } catch (e) { Object.defineProperty(BABYLON, k, { value: v, writable: true, configurable: true }); } };
  let current = null;   // the engine whose context owns textures created without an engine argument

  function check(ctx, rc, what) {
    if (typeof rc === 'number' && rc !== 0) report(what + ': ' + (ERR[rc] || rc) + ' ' + addon.pt_last_error(ctx));
    return rc;
  }
  function ctxOf(sceneOrEngine) {
    if (sceneOrEngine && sceneOrEngine._pt) return sceneOrEngine._pt;
    if (sceneOrEngine && sceneOrEngine.getEngine && sceneOrEngine.getEngine()._pt) return sceneOrEngine.getEngine()._pt;
    return current._pt;
  }

  class Engine extends RealNull {
    constructor(canvas, antialias, options) {
      const w = (canvas && canvas.width) || opts.width, h = (canvas && canvas.height) || opts.height;
      super({ renderWidth: w, renderHeight: h, textureSize: 512, deterministicLockstep: false, lockstepMaxSteps: 1 });
      // the devices of the context: opts.devices, else PT_DEVICES ("0,1,2,3"; a device may repeat),
      // else opts.device - with several, every draw fans out over them inside libpt (pt.h)
      const devs = opts.devices || (process.env.PT_DEVICES ? process.env.PT_DEVICES.split(',').map((d) => parseInt(d, 10)) : null);
      const c = devs ? addon.pt_ctx_create_devices(devs) : addon.pt_ctx_create(opts.device);
      if (typeof c === 'number') throw new Error('pt_ctx_create: ' + (ERR[c] || c));
      this._pt = c;
      this._renderLoop = null;
      this.isPointerLock = false;
      addon.pt_canvas_resize(c, w, h);
      current = this;
    }
    runRenderLoop(fn) { this._renderLoop = fn; }
    // the browser calls the loop from requestAnimationFrame; a Node host steps it explicitly
    stepFrame() { if (this._renderLoop) this._renderLoop(); }
    enterPointerlock() {}
    exitPointerlock() {}
    setHardwareScalingLevel(l) { this._scaling = l; }
    getDeltaTime() { return opts.deltaTimeMs || 1000 / 60; }
    resize() { addon.pt_canvas_resize(this._pt, this.getRenderWidth(), this.getRenderHeight()); }
    readCanvas() {
      const out = new Uint8Array(this.getRenderWidth() * this.getRenderHeight() * 4);
      check(this._pt, addon.pt_read_pixels(this._pt, null, out), 'readPixels');
      return out;
    }
    dispose() { if (this._pt) { addon.pt_ctx_destroy(this._pt); this._pt = null; } super.dispose(); }
  }

  class RenderTargetTexture {
    constructor(name, size, scene) {
      this.name = name;
      this._ctx = ctxOf(scene);
      const h = addon.pt_render_target_create(this._ctx, size.width, size.height);
      if (typeof h === 'number') throw new Error('RenderTargetTexture: ' + (ERR[h] || h));
      this._pt = label(h, name);
    }
    getSize() { const s = addon.pt_texture_size(this._pt); return { width: s[0], height: s[1] }; }
    resize(size) { check(this._ctx, addon.pt_render_target_resize(this._pt, size.width, size.height), 'resize'); }
    readPixels() {
      const s = this.getSize(), out = new Float32Array(s.width * s.height * 4);
      check(this._ctx, addon.pt_read_pixels(this._ctx, this._pt, out), 'readPixels');
      return out;
    }
    dispose() { if (this._pt) addon.pt_texture_destroy(this._pt); this._pt = null; }
  }

  const RawTexture = {
    CreateRGBATexture(data, w, h, scene, generateMipMaps, invertY, samplingMode, type) {
      const ctx = ctxOf(scene);
      const t = { name: 'RawTexture', _ctx: ctx };
      const sampling = samplingMode === undefined ? 3 : samplingMode;
      const handle = type === TEXTURETYPE_UNSIGNED_BYTE || data instanceof Uint8Array
        ? addon.pt_texture_create_rgba8(ctx, w, h, data, sampling, invertY ? 1 : 0)
        : addon.pt_texture_create_rgba32f(ctx, w, h, data, sampling, invertY ? 1 : 0);
      if (typeof handle === 'number') { report('CreateRGBATexture: ' + (ERR[handle] || handle)); return null; }
      t._pt = label(handle, 'RawTexture');
      t.dispose = () => { if (t._pt) addon.pt_texture_destroy(t._pt); t._pt = null; };
      return t;
    },
  };

  function adoptForeign(ctx, t) {
    t._ptForeign = null;
    const bytes = t._buffer;
    if (!bytes || typeof bytes === 'string') return;
    try {
      const img = decodeImage(bytes, addon);
      const sm = typeof t.samplingMode === 'number' ? t.samplingMode : 3;
      const h = addon.pt_texture_create_rgba8(ctx, img.width, img.height, img.data, sm, t._invertY ? 1 : 0);
      if (typeof h !== 'number') t._ptForeign = label(h, t.name || t.url || 'texture');
    } catch (e) {
      report('texture ' + (t.name || t.url) + ': ' + e.message + ' (left unbound)');
    }
  }

  class Texture {
    // new Texture(url, scene, noMipmap, invertY, samplingMode, onLoad) or, as the glTF loader calls
    // it, new Texture(null, scene, { invertY, samplingMode, onLoad, ... }) then updateURL(url, bytes)
    constructor(url, scene, noMipmap, invertY, samplingMode, onLoad) {
      if (noMipmap && typeof noMipmap === 'object') {
        const o = noMipmap;
        invertY = o.invertY; samplingMode = o.samplingMode; onLoad = o.onLoad;
      }
      this._name = url || '';
      this._ctx = ctxOf(scene);
      this._pt = null;
      this._size = { width: 0, height: 0 };
      this._pixels = null;
      this._invertY = invertY === undefined ? true : !!invertY;
      this._sampling = samplingMode === undefined ? 3 : samplingMode;
      this._onLoad = onLoad;
      if (url === null || url === undefined) return;   // bytes follow through updateURL
      // page-relative URLs resolve against baseDir, then the extra opts.assetDirs
      const dirs = [opts.baseDir].concat(opts.assetDirs || []);
      const file = path.isAbsolute(url) ? url
        : (dirs.map((d) => path.join(d, url)).find((f) => fs.existsSync(f)) || path.join(opts.baseDir, url));
      if (/\.hdr$/i.test(url)) {
        // an environment: decoded on the host, handed back through readPixels(); the setup script
        // re-uploads it as a RawTexture (so nothing is bound here)
        try {
          const img = decodeHDR(fs.readFileSync(file));
          this._size = { width: img.width, height: img.height };
          this._pixels = img.data;
          if (onLoad) setImmediate(onLoad);
        } catch (e) {
          report('Texture(' + url + '): ' + e.message + ' (not loaded)');
        }
        return;
      }
      let bytes;
      try { bytes = fs.readFileSync(file); } catch (e) { report('Texture(' + url + '): ' + e.message + ' (left unbound)'); return; }
      this._upload(bytes, url);
    }
    // the glTF loader's path: the image file's bytes (Babylon's Texture.updateURL(url, buffer))
    updateURL(url, buffer) {
      if (!this._name || this._name.startsWith('data:')) this._name = url;
      if (this._pt) { addon.pt_texture_destroy(this._pt); this._pt = null; }
      if (buffer) this._upload(buffer, url);
      else report('Texture.updateURL(' + url + '): no image bytes (left unbound)');
    }
    _upload(bytes, what) {
      try {
        const img = decodeImage(bytes, addon);
        this._size = { width: img.width, height: img.height };
        const h = addon.pt_texture_create_rgba8(this._ctx, img.width, img.height, img.data, this._sampling, this._invertY ? 1 : 0);
        if (typeof h !== 'number') this._pt = label(h, this._name || what);
        if (this._onLoad) setImmediate(this._onLoad);
      } catch (e) {
        report('Texture(' + what + '): ' + e.message + ' (left unbound)');
      }
    }
    get name() { return this._name; }
    set name(v) { this._name = v; if (this._pt) label(this._pt, v); }
    getSize() { return this._size; }
    readPixels() { return Promise.resolve(this._pixels); }
    dispose() { if (this._pt) addon.pt_texture_destroy(this._pt); this._pt = null; }
  }

  class Effect {
    constructor(ctx, handle) { this._ctx = ctx; this._pt = handle; }
    isReady() { return this._pt !== null; }
    _f(name, arr) { if (this._pt) check(this._ctx, addon.pt_set_float(this._pt, name, arr), 'set ' + name); return this; }
    setFloat(n, v) { return this._f(n, [v]); }
    setFloat2(n, a, b) { return this._f(n, [a, b]); }
    setFloat3(n, a, b, c) { return this._f(n, [a, b, c]); }
    setFloat4(n, a, b, c, d) { return this._f(n, [a, b, c, d]); }
    setVector2(n, v) { return this._f(n, [v.x, v.y]); }
    setVector3(n, v) { return this._f(n, [v.x, v.y, v.z]); }
    setMatrix(n, m) { return this._f(n, Array.from(m.m !== undefined ? m.m : m.toArray())); }
    setInt(n, v) { if (this._pt) check(this._ctx, addon.pt_set_int(this._pt, n, v | 0), 'setInt ' + n); return this; }
    setBool(n, v) { return this.setInt(n, v ? 1 : 0); }
    setTexture(n, t) {
      // an unloaded Babylon texture (null / undefined, e.g. a model without albedo map) binds
      // nothing; a texture Babylon itself created (the glTF loader's PBR maps) is uploaded once,
      // from the image bytes it keeps (Texture.updateURL(url, buffer))
      if (t && !t._pt && t._ptForeign === undefined) adoptForeign(this._ctx, t);
      const h = t ? (t._pt || t._ptForeign || null) : null;
      if (this._pt) check(this._ctx, addon.pt_set_texture(this._pt, n, h), 'setTexture ' + n);
      return this;
    }
  }

  class EffectWrapper {
    constructor(o) {
      this.name = o.name;
      const ctx = ctxOf(o.engine);
      // o.ptProgram (extension): name the program directly when the GLSL text is not at hand
      const h = o.ptProgram
        ? addon.pt_effect_create_program(ctx, o.ptProgram, o.uniformNames || [], o.samplerNames || [])
        : addon.pt_effect_create(ctx, o.fragmentShader || '', o.uniformNames || [], o.samplerNames || []);
      label(h, o.name);
      if (typeof h === 'number') report('EffectWrapper(' + o.name + '): ' + (ERR[h] || h) + ' ' + addon.pt_last_error(ctx));
      this.effect = new Effect(ctx, typeof h === 'number' ? null : h);
      this._observers = [];
      this.onApplyObservable = { add: (f) => { this._observers.push(f); return f; }, clear: () => { this._observers = []; } };
    }
    dispose() { if (this.effect._pt) addon.pt_effect_destroy(this.effect._pt); this.effect._pt = null; }
  }

  class EffectRenderer {
    constructor(engine) { this.engine = engine; }
    // Babylon skips a non-ready effect silently; so does this
    render(wrapper, target) {
      if (!wrapper.effect.isReady()) return;
      wrapper._observers.forEach((f) => f());
      check(wrapper.effect._ctx, addon.pt_render(wrapper.effect._pt, target ? target._pt : null), 'render ' + wrapper.name);
    }
    dispose() {}
  }

  set('Engine', Engine);
  set('RenderTargetTexture', RenderTargetTexture);
  set('RawTexture', RawTexture);
  set('Texture', Texture);
  set('EffectWrapper', EffectWrapper);
  set('EffectRenderer', EffectRenderer);
  return { addon, Engine, decodePNG, decodeHDR, decodeImage, nativeBVH: (device) => nativeBVH(addon, device) };
}

// BVH_Build_Iterative(workList, aabb_array) (js/BVH_Fast_Builder.js:320-406) over libpt's native
// builder (same tree, same bits); with a device number, over the device build (pt_bvh_build_gpu,
// same bits again). A host installs it after loading BVH_Fast_Builder.js:
//   globalThis.BVH_Build_Iterative = require('.../babylon_pt.js').nativeBVH(addon[, device]);
function nativeBVH(addon, device) {
  return function BVH_Build_Iterative(workList, aabbArray) {
    const n = workList.length;
    const out = new Float32Array(8 * (2 * n - 1));
    const work = Uint32Array.from(workList);
    const rc = device === undefined || device === null
      ? addon.pt_bvh_build(aabbArray.subarray(0, 9 * n), work, out)
      : addon.pt_bvh_build_gpu(device, aabbArray, work, out);
    if (rc < 0) throw new Error('pt_bvh_build: ' + (ERR[rc] || rc));
    aabbArray.set(out, 0);
  };
}

module.exports = { install, decodePNG, decodeHDR, decodeImage, nativeBVH, loadAddon };
