# Host sanitizer build of the CPU twin (TEST INFRASTRUCTURE ONLY; SURVEY.md §5,
# tests/test_sanitizers.py): zb_oracle.c (fp32, no OpenMP) + the stepping driver.
#   make -C oracle -f asan.mk
CC ?= gcc
SAN = -fsanitize=address,undefined -fsanitize=bounds -fno-sanitize-recover=all -fno-omit-frame-pointer
_asan/zb_oracle_selftest: zb_oracle.c zb_oracle_selftest.c ../include/zbot_model.h ../include/zbot_layout.h
	@mkdir -p _asan
	$(CC) -std=c11 -O1 -g $(SAN) -ffp-contract=off -Wall -Wno-unused-function -Wno-unknown-pragmas -I../include -o $@ zb_oracle.c zb_oracle_selftest.c -lm
.DEFAULT_GOAL := _asan/zb_oracle_selftest
