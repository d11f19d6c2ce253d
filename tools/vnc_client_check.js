// Drives the browser VNC client core (web/vnc.js) from Node against a running RFB server over
// plain TCP; used by tests/test_vnc_client.py.  Usage:
//   node tools/vnc_client_check.js PORT PASSWORD UPDATES
// Prints one JSON line: size, desktop name, updates, md5 of the RGBA framebuffer after each
// update; after the first update it sends a pointer event, a key press and cut text.
"use strict";
const net = require("net");
const crypto = require("crypto");
const path = require("path");
const { RfbClient } = require(path.join(__dirname, "..", "web", "vnc.js"));

const [port, password, updates] = [Number(process.argv[2]), process.argv[3], Number(process.argv[4] || 1)];
const sock = net.connect(port, "127.0.0.1");
const digests = [];
let client;
client = new RfbClient((u8) => sock.write(Buffer.from(u8)), {
  password,
  onUpdate: () => {
    digests.push(crypto.createHash("md5").update(Buffer.from(client.fb)).digest("hex"));
    if (client.updates === 1) { client.pointer(12, 34, 1); client.key(0x61, true); client.cutText("hi there"); }
    if (client.updates >= updates) {
      console.log(JSON.stringify({ width: client.width, height: client.height, name: client.name, updates: client.updates, digests }));
      sock.destroy();
      process.exit(0);
    }
  },
});
sock.on("data", (b) => client.feed(new Uint8Array(b.buffer, b.byteOffset, b.length)));
sock.on("close", () => client.close());
client.run().catch((e) => { console.log(JSON.stringify({ error: String(e.message || e) })); process.exit(1); });
setTimeout(() => { console.log(JSON.stringify({ error: "timeout", updates: client.updates })); process.exit(2); }, 20000);
