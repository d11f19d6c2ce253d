/* Hardware probe: does this amdgpu device expose a VCN
 * encoder, and which codecs does the kernel driver advertise for encode/decode?
 * Also reports the render node, device id and whether the IP has display rings.
 * Built with: cc vcn_caps.c -I/usr/include/libdrm -ldrm_amdgpu -ldrm */
#include <amdgpu.h>
#include <amdgpu_drm.h>
#include <fcntl.h>
#include <stdio.h>
#include <unistd.h>
#include <dirent.h>
#include <string.h>

static const char *codec_name[] = {"mpeg2", "mpeg4", "vc1", "h264", "hevc", "jpeg", "vp9", "av1"};

static void dump_caps(amdgpu_device_handle dev, unsigned which, const char *tag) {
    struct drm_amdgpu_info_video_caps caps;
    memset(&caps, 0, sizeof caps);
    int r = amdgpu_query_video_caps_info(dev, which, sizeof caps, &caps);
    printf("  \"%s\": {\"ret\": %d", tag, r);
    for (int i = 0; i < AMDGPU_INFO_VIDEO_CAPS_CODEC_IDX_COUNT; ++i) {
        struct drm_amdgpu_info_video_codec_info *c = &caps.codec_info[i];
        printf(", \"%s\": {\"valid\": %u, \"max_w\": %u, \"max_h\": %u, \"max_level\": %u}", codec_name[i],
               c->valid, c->max_width, c->max_height, c->max_level);
    }
    printf("},\n");
}

static void dump_ip(amdgpu_device_handle dev, unsigned type, const char *tag) {
    struct drm_amdgpu_info_hw_ip ip;
    memset(&ip, 0, sizeof ip);
    unsigned count = 0;
    int rc = amdgpu_query_hw_ip_count(dev, type, &count);
    int r = amdgpu_query_hw_ip_info(dev, type, 0, &ip);
    printf("  \"ip_%s\": {\"count_ret\": %d, \"count\": %u, \"ret\": %d, \"ver\": \"%u.%u\", \"rings\": %u},\n", tag, rc,
           count, r, ip.hw_ip_version_major, ip.hw_ip_version_minor, ip.available_rings);
}

int main(void) {
    DIR *d = opendir("/dev/dri");
    if (!d) { printf("{\"error\": \"no /dev/dri\"}\n"); return 0; }
    struct dirent *e;
    printf("[\n");
    while ((e = readdir(d))) {
        if (strncmp(e->d_name, "renderD", 7)) continue;
        char path[256];
        snprintf(path, sizeof path, "/dev/dri/%s", e->d_name);
        int fd = open(path, O_RDWR);
        if (fd < 0) { printf("{\"node\": \"%s\", \"error\": \"open failed\"},\n", path); continue; }
        uint32_t maj, min;
        amdgpu_device_handle dev;
        if (amdgpu_device_initialize(fd, &maj, &min, &dev)) { printf("{\"node\": \"%s\", \"error\": \"init\"},\n", path); close(fd); continue; }
        struct amdgpu_gpu_info gi;
        amdgpu_query_gpu_info(dev, &gi);
        printf("{ \"node\": \"%s\", \"asic_id\": \"0x%x\", \"family\": %u, \"chip_ext_rev\": %u, \"num_se\": %u,\n", path, gi.asic_id,
               gi.family_id, gi.chip_external_rev, gi.num_shader_engines);
        const char *name = amdgpu_get_marketing_name(dev);
        printf("  \"marketing\": \"%s\",\n", name ? name : "?");
        dump_ip(dev, AMDGPU_HW_IP_GFX, "gfx");
        dump_ip(dev, AMDGPU_HW_IP_COMPUTE, "compute");
        dump_ip(dev, AMDGPU_HW_IP_VCN_DEC, "vcn_dec");
        dump_ip(dev, AMDGPU_HW_IP_VCN_ENC, "vcn_enc");
        dump_ip(dev, AMDGPU_HW_IP_VCN_JPEG, "vcn_jpeg");
        dump_ip(dev, AMDGPU_HW_IP_UVD, "uvd");
        dump_ip(dev, AMDGPU_HW_IP_VCE, "vce");
        dump_caps(dev, AMDGPU_INFO_VIDEO_CAPS_DECODE, "decode");
        dump_caps(dev, AMDGPU_INFO_VIDEO_CAPS_ENCODE, "encode");
        printf("  \"end\": 0},\n");
        amdgpu_device_deinitialize(dev);
        close(fd);
    }
    printf("{}]\n");
    closedir(d);
    return 0;
}
