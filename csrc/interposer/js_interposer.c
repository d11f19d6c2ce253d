// Joystick interposer (replaces selkies' joystick_interposer.so that the
// reference preloads, Dockerfile:473-476).  LD_PRELOAD'ed into desktop apps/games:
//
//   open("/dev/input/jsN")  ->  connect(AF_UNIX, "$MXDESK_JS_DIR/mxdesk_jsN.sock")
//
// The mxdesk server (mxdesk/server/gamepad.py) owns the sockets.  On connect it sends one
// config record (name, axis/button counts and maps), then a stream of Linux `struct
// js_event` (8 bytes) generated from the browser's Gamepad API.  The app reads js_events
// straight from the socket; the joystick ioctls (JSIOCGVERSION/AXES/BUTTONS/NAME/AXMAP/
// BTNMAP, CORR) are answered from the config record.  No kernel device or uinput access is
// needed, so it works in an unprivileged container.
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/joystick.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#define MX_MAX_JS 4
#define MX_NAME_LEN 128

// Wire format of the config record (little-endian, packed); mirrored by gamepad.py.
struct mx_js_config {
    char name[MX_NAME_LEN];
    uint16_t num_buttons;
    uint8_t num_axes;
    uint8_t pad;
    uint16_t btn_map[KEY_MAX - BTN_MISC + 1];
    uint8_t axes_map[ABS_CNT];
} __attribute__((packed));

struct mx_js {
    int fd;  // socket fd returned to the app, -1 if unused
    struct mx_js_config cfg;
};

static struct mx_js g_js[MX_MAX_JS] = {{-1}, {-1}, {-1}, {-1}};
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

typedef int (*open_fn)(const char*, int, ...);
typedef int (*openat_fn)(int, const char*, int, ...);
typedef int (*ioctl_fn)(int, unsigned long, ...);
typedef int (*close_fn)(int);

static void* real(const char* sym) {
    void* p = dlsym(RTLD_NEXT, sym);
    if (!p) fprintf(stderr, "mxdesk-js: dlsym(%s) failed\n", sym);
    return p;
}

// Returns the joystick index for "/dev/input/jsN", else -1.
static int js_index(const char* path) {
    static const char pre[] = "/dev/input/js";
    if (!path || strncmp(path, pre, sizeof(pre) - 1) != 0) return -1;
    const char* n = path + sizeof(pre) - 1;
    if (n[0] < '0' || n[0] > '9' || n[1] != '\0') return -1;
    const int i = n[0] - '0';
    return i < MX_MAX_JS ? i : -1;
}

static int read_full(int fd, void* buf, size_t n) {
    size_t got = 0;
    while (got < n) {
        const ssize_t r = read(fd, (char*)buf + got, n - got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return -1;
        got += (size_t)r;
    }
    return 0;
}

static int js_connect(int idx, int flags) {
    const char* dir = getenv("MXDESK_JS_DIR");
    struct sockaddr_un sa;
    memset(&sa, 0, sizeof(sa));
    sa.sun_family = AF_UNIX;
    snprintf(sa.sun_path, sizeof(sa.sun_path), "%s/mxdesk_js%d.sock", dir ? dir : "/tmp", idx);
    const int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    if (connect(fd, (struct sockaddr*)&sa, sizeof(sa)) != 0) {
        close(fd);
        errno = ENOENT;  // behave like an absent device
        return -1;
    }
    struct mx_js_config cfg;
    if (read_full(fd, &cfg, sizeof(cfg)) != 0) {
        close(fd);
        errno = EIO;
        return -1;
    }
    cfg.name[MX_NAME_LEN - 1] = '\0';
    if (flags & O_NONBLOCK) fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    pthread_mutex_lock(&g_lock);
    g_js[idx].fd = fd;
    g_js[idx].cfg = cfg;
    pthread_mutex_unlock(&g_lock);
    return fd;
}

static struct mx_js* js_of_fd(int fd) {
    for (int i = 0; i < MX_MAX_JS; ++i)
        if (g_js[i].fd == fd && fd >= 0) return &g_js[i];
    return NULL;
}

#define OPEN_MODE(flags, mode)                \
    mode_t mode = 0;                          \
    if ((flags) & (O_CREAT | O_TMPFILE)) {    \
        va_list ap;                           \
        va_start(ap, flags);                  \
        mode = (mode_t)va_arg(ap, int);       \
        va_end(ap);                           \
    }

int open(const char* path, int flags, ...) {
    OPEN_MODE(flags, mode);
    const int idx = js_index(path);
    if (idx >= 0) return js_connect(idx, flags);
    static open_fn fn;
    if (!fn) fn = (open_fn)real("open");
    return fn(path, flags, mode);
}

int open64(const char* path, int flags, ...) {
    OPEN_MODE(flags, mode);
    const int idx = js_index(path);
    if (idx >= 0) return js_connect(idx, flags);
    static open_fn fn;
    if (!fn) fn = (open_fn)real("open64");
    return fn(path, flags, mode);
}

int openat(int dirfd, const char* path, int flags, ...) {
    OPEN_MODE(flags, mode);
    const int idx = js_index(path);
    if (idx >= 0) return js_connect(idx, flags);
    static openat_fn fn;
    if (!fn) fn = (openat_fn)real("openat");
    return fn(dirfd, path, flags, mode);
}

int openat64(int dirfd, const char* path, int flags, ...) {
    OPEN_MODE(flags, mode);
    const int idx = js_index(path);
    if (idx >= 0) return js_connect(idx, flags);
    static openat_fn fn;
    if (!fn) fn = (openat_fn)real("openat64");
    return fn(dirfd, path, flags, mode);
}

int close(int fd) {
    pthread_mutex_lock(&g_lock);
    struct mx_js* js = js_of_fd(fd);
    if (js) js->fd = -1;
    pthread_mutex_unlock(&g_lock);
    static close_fn fn;
    if (!fn) fn = (close_fn)real("close");
    return fn(fd);
}

int ioctl(int fd, unsigned long req, ...) {
    va_list ap;
    va_start(ap, req);
    void* arg = va_arg(ap, void*);
    va_end(ap);
    pthread_mutex_lock(&g_lock);
    struct mx_js* js = js_of_fd(fd);
    struct mx_js_config cfg;
    if (js) cfg = js->cfg;
    pthread_mutex_unlock(&g_lock);
    if (!js) {
        static ioctl_fn fn;
        if (!fn) fn = (ioctl_fn)real("ioctl");
        return fn(fd, req, arg);
    }
    switch (_IOC_TYPE(req) == 'j' ? _IOC_NR(req) : -1) {
        case 0x01:  // JSIOCGVERSION
            *(uint32_t*)arg = JS_VERSION;
            return 0;
        case 0x11:  // JSIOCGAXES
            *(uint8_t*)arg = cfg.num_axes;
            return 0;
        case 0x12:  // JSIOCGBUTTONS
            *(uint8_t*)arg = (uint8_t)cfg.num_buttons;
            return 0;
        case 0x13: {  // JSIOCGNAME(len)
            const size_t len = _IOC_SIZE(req);
            const size_t n = strnlen(cfg.name, MX_NAME_LEN - 1);
            if (len == 0) return 0;
            memcpy(arg, cfg.name, n < len ? n + 1 : len);
            ((char*)arg)[len - 1] = '\0';
            return (int)(n < len ? n + 1 : len);
        }
        case 0x32:  // JSIOCGAXMAP
            memcpy(arg, cfg.axes_map, sizeof(cfg.axes_map));
            return 0;
        case 0x34:  // JSIOCGBTNMAP
            memcpy(arg, cfg.btn_map, sizeof(cfg.btn_map));
            return 0;
        case 0x21:  // JSIOCSCORR
        case 0x31:  // JSIOCSAXMAP
        case 0x33:  // JSIOCSBTNMAP
            return 0;
        case 0x22:  // JSIOCGCORR
            memset(arg, 0, sizeof(struct js_corr) * (cfg.num_axes ? cfg.num_axes : 1));
            return 0;
        default:
            errno = ENOTTY;
            return -1;
    }
}
