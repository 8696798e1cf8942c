set -u
bash tools/gpu_session.sh tests multi4 smoke
