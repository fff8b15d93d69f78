'use strict';
// PropertyBag with the reference's surface (PropertyBag.js:1-16): a
// `properties` list, one writable field per property, and an EventTarget-like
// addEventListener / dispatchEvent for the 'change' events the UI sends
// (Application.js:128-139). Node 12 has no global EventTarget/CustomEvent, so
// a minimal one is provided here.

class Evented {
  constructor() {
    this._listeners = new Map();
  }

  addEventListener(type, fn) {
    if (!this._listeners.has(type)) this._listeners.set(type, []);
    this._listeners.get(type).push(fn);
  }

  removeEventListener(type, fn) {
    const l = this._listeners.get(type);
    if (l) this._listeners.set(type, l.filter(f => f !== fn));
  }

  dispatchEvent(event) {
    const l = this._listeners.get(event.type) || [];
    for (const fn of l.slice()) fn.call(this, event);
    return true;
  }
}

function changeEvent(name, value) {
  return { type: 'change', detail: { name, value } };
}

class PropertyBag extends Evented {
  constructor() {
    super();
    this.properties = [];
  }

  registerProperties(properties) {
    this.properties.push(...properties);
    for (const property of properties) {
      this[property.name] = property.value;
    }
  }

  // UI-style property edit: assign, then announce (Application.js:131-139)
  setProperty(name, value) {
    this[name] = value;
    this.dispatchEvent(changeEvent(name, value));
  }
}

module.exports = { PropertyBag, Evented, changeEvent };
