set -o pipefail
PMC="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM" tools/prof_pmc.sh pmc_hevc4k --codec hevc --width 3840 --height 2160 --bitrate-kbps 25000 --steps 20 --warmup 3 --quality-probe 0 --density-probe 0
