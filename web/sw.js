// PWA service worker (reference: selkies-gstreamer-entrypoint.sh:37-38 templates PWA_CACHE)
const CACHE = "mxdesk-pwa-v1";
self.addEventListener("install", (e) => e.waitUntil(caches.open(CACHE).then((c) => c.addAll(["index.html", "client.js"]))));
self.addEventListener("fetch", (e) => {
  if (e.request.method !== "GET" || new URL(e.request.url).pathname.startsWith("/mxws")) return;
  e.respondWith(fetch(e.request).catch(() => caches.match(e.request)));
});
