#!/bin/bash
# round 6: the whole GPU suite + smoke, then the driver's default bench line
export TMPDIR=/tmp
bash tools/gpu_task.sh suite r6suite && bash tools/gpu_task.sh bench r6bench
