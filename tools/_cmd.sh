set -u
V=pypanadapter_amd/lib/variants
AB_REPS=2 bash tools/ab.sh r03f_ko base=default ko39=$V/libzfft_ko39.so ko24=$V/libzfft_ko24.so ko63=$V/libzfft_ko63.so ko7=$V/libzfft_ko7.so
