#!/usr/bin/env perl
# Test helper for tests/test_perl_xs.py: drives the Perl side of the XS binding
# (perl/lib/Prgpu.pm) on a chunk given as JSON {reads, alns, params}.
#
#   perl_cns_helper.pl pack IN.json  -> {field: hex of the packed pr_cns_batch buffer}
#   perl_cns_helper.pl run  IN.json  -> [{id, status, seq, qual, trace, cigar, chim}] (GPU)
use strict;
use warnings;
use FindBin;
use lib "$FindBin::RealBin/../perl/lib";
use JSON::PP;
use Prgpu;

my ($mode, $file) = @ARGV;
open my $fh, '<', $file or die "$file: $!\n";
my $in = decode_json(do { local $/; <$fh> });
close $fh;
my $json = JSON::PP->new->canonical;

if ($mode eq 'pack') {
    my $b = Prgpu::pack_chunk($in->{reads}, $in->{alns});
    my %hex = map { $_ => ($_ eq 'n_lr' ? $b->{$_} : unpack('H*', $b->{$_})) } keys %$b;
    print $json->encode(\%hex), "\n";
} elsif ($mode eq 'run') {
    my $ctx = Prgpu::Context->new(0);
    my @res = Prgpu::run_chunk($ctx, $in->{params}, $in->{reads}, $in->{alns});
    for my $r (@res) { $r->{chim_lines} = [Prgpu::chim_lines($r)]; $r->{fastq} = $r->{status} ? '' : Prgpu::fastq($r) }
    print $json->encode(\@res), "\n";
} else {
    die "usage: perl_cns_helper.pl pack|run IN.json\n";
}
