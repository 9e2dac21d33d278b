for r in 1 2; do for v in 1 0; do
PFM_FFN_FUSED=$v python bench.py --exact-steps 0 --cpu-utts 0 --stream-chunks 0 --punc-steps 0 --long-audio-s 0 --steps 5 --sv-steps 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('FFN_FUSED=$v', d['ms_per_step'], d['sensevoice']['ms_per_step'])"
done; done
