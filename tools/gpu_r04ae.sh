bash tools/profile_fast.sh r04ae_fast
