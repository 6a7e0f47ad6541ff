#!/bin/bash
# Reference download_models.sh fetches models.zip (raft-things/-sintel/-kitti/-chairs/-small .pth)
# from Dropbox.  This environment has no network: place the reference .pth files under models/
# yourself.  They load unchanged (DataParallel 'module.' prefix handled):
#   python evaluate.py --model models/raft-things.pth --dataset sintel --mixed_precision
set -e
mkdir -p models
if [[ -n "${RAFT_MODELS_ZIP:-}" && -f "${RAFT_MODELS_ZIP}" ]]; then
  python -c "import zipfile,sys; zipfile.ZipFile(sys.argv[1]).extractall('.')" "${RAFT_MODELS_ZIP}"
fi
ls -la models
