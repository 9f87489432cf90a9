#!/bin/bash
# Fetch the pretrained RAFT checkpoints published with the original RAFT release
# (raft-things / chairs / sintel / kitti / small .pth).  They are in the reference's
# DataParallel format and load directly with --model / --restore_ckpt.
# Needs network access (not available inside the build sandbox).
set -e
URL=${RAFT_MODELS_URL:-https://dl.dropboxusercontent.com/s/4j4z58wuv8o0mfz/models.zip}
wget -O models.zip "$URL"
unzip -o models.zip
