#!/usr/bin/env perl
# Golden-vector generator for the trim-window and quality-run restatements.
#
# Loads the REFERENCE module Fastq::Seq from the read-only checkout (default
# /root/reference/lib) and calls it per case:
#   WIN  cases: Fastq::Seq::qual_window (lib/Fastq/Seq.pm:1064-1160) with the
#               class globals set per case (Qual_window_size / _min_score_soft /
#               _min_score_hard / _min_stretch_length).
#   MASK cases: Fastq::Seq::qual_lcs (Seq.pm:709-717), the HCR search the
#               masking step starts from, with the range and minimum length
#               of the case (sam2cns:432-434 layout: min = mask_min + 2*reduce).
#               Qual_lcs_regex is assigned per case: the setters build it with
#               qr//o, which keeps the first pattern for the whole process.
#
# Usage: perl gen_seqfilter_golden.pl cases.txt > expected.txt
# Only this container runs it; its outputs are committed as fixtures.
use strict;
use warnings;

BEGIN {
    my $ref = $ENV{PROOVREAD_REFERENCE} || '/root/reference';
    unshift @INC, "$ref/lib";
}
use Fastq::Seq;

$SIG{__WARN__} = sub { };

sub pairs { join(' ', map { "$_->[0],$_->[1]" } @_) }

while (my $line = <>) {
    chomp $line;
    next unless length $line;
    my @f = split /\t/, $line, -1;
    my $kind = shift @f;
    if ($kind eq 'WIN') {
        my ($size, $soft, $hard, $minl, $q) = @f;
        Fastq::Seq->Qual_window_size($size);
        Fastq::Seq->Qual_window_min_score_soft($soft);
        Fastq::Seq->Qual_window_min_score_hard($hard);
        Fastq::Seq->Qual_window_min_stretch_length($minl);
        my $fq = Fastq::Seq->new(seq_head => '@r', seq => 'A' x length($q), qual_head => '+', qual => $q,
                                 phred_offset => 33);
        my @w = $fq->qual_window();
        print "WIN\t", pairs(@w), "\n";
    } elsif ($kind eq 'MASK') {
        my ($pmin, $pmax, $mmin, $umin, $red, $er, $q) = @f;
        my $range = join('', map { chr($_ + 33) } $pmin .. $pmax);
        $range =~ s/([\\\^\-\[\]])/\\$1/g;
        my $minlen = $mmin + 2 * $red;
        $Fastq::Seq::Qual_lcs_regex = qr/([$range]{$minlen,})/;
        my $fq = Fastq::Seq->new(seq_head => '@r', seq => 'A' x length($q), qual_head => '+', qual => $q,
                                 phred_offset => 33);
        my @h = $fq->qual_lcs();
        print "MASK\t", pairs(@h), "\n";
    } else {
        die "bad case line: $kind";
    }
}
