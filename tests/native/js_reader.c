// Test "game": opens /dev/input/js0 like SDL/joydev users do, queries it with the joystick
// ioctls and prints N events.  Run under LD_PRELOAD=libmxjs_interposer.so.
#include <fcntl.h>
#include <linux/joystick.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/ioctl.h>
#include <unistd.h>

int main(int argc, char** argv) {
    const int want = argc > 1 ? atoi(argv[1]) : 4;
    const int fd = open("/dev/input/js0", O_RDONLY);
    if (fd < 0) {
        perror("open");
        return 2;
    }
    unsigned int ver = 0;
    unsigned char axes = 0, buttons = 0;
    char name[128] = {0};
    __u16 btnmap[KEY_MAX - BTN_MISC + 1];
    __u8 axmap[ABS_CNT];
    if (ioctl(fd, JSIOCGVERSION, &ver) || ioctl(fd, JSIOCGAXES, &axes) || ioctl(fd, JSIOCGBUTTONS, &buttons) ||
        ioctl(fd, JSIOCGNAME(sizeof(name)), name) < 0 || ioctl(fd, JSIOCGBTNMAP, btnmap) ||
        ioctl(fd, JSIOCGAXMAP, axmap)) {
        perror("ioctl");
        return 3;
    }
    printf("version=%06x axes=%d buttons=%d name=%s btn0=%#x ax2=%d\n", ver, axes, buttons, name, btnmap[0], axmap[2]);
    int got = 0;
    struct js_event e;
    while (got < want && read(fd, &e, sizeof(e)) == (ssize_t)sizeof(e)) {
        if (e.type & JS_EVENT_INIT) continue;
        printf("event type=%d number=%d value=%d\n", e.type, e.number, e.value);
        ++got;
    }
    fflush(stdout);
    close(fd);
    return got == want ? 0 : 4;
}
