#!/bin/bash
# Bench configs 4 and 2 back to back on one box, printing each run's ms/frame and the frame
# renderer's timed choices (the sequence behind the timed-choice margin, docs/ROUND_LOG.md 5).
set -e
for c in 4 2 2 4 2; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/seq_$c.json 2>/dev/null
  python -c "import json; d=json.loads([l for l in open('gpurun_out/seq_$c.json').read().splitlines() if l.startswith('{')][-1]); print('cfg $c', d['ms_per_step'], d['frame_ms_events'], d.get('timed_choices'), d['overlapped_frames'], d.get('at_720p',{}).get('ms_per_frame'), d.get('at_720p',{}).get('in_flight'))"
done
