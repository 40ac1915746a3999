#!/usr/bin/env perl
# Golden-vector generator for the consensus stage.
#
# Runs the REFERENCE consensus engine (Sam::Seq / Sam::Alignment / Fastq::Seq
# from the read-only reference checkout, default /root/reference/lib) on every
# case of a case file (tests/golden/casefmt.py) and prints the expected
# outputs.  It reproduces what bin/bam2cns does per long read
# (bam2cns:227-237 class setup, 332-365 per-read loop, 375-455
# generate_consensus, 461-491 detect_chimera) without samtools: alignments are
# fed from SAM text in the case's (BAM) order.
#
# Determinism (SURVEY.md §8c): run with PERL_HASH_SEED=0 PERL_PERTURB_KEYS=0
# and Sam::Seq::alns is overridden to return alignments in ascending internal
# id (arrival) order, the canonical order the C oracle and the GPU use.
#
# Usage: perl gen_cns_golden.pl cases.txt > expected.txt
# Only this container runs it; its outputs are committed as fixtures.
use strict;
use warnings;

BEGIN {
    my $ref = $ENV{PROOVREAD_REFERENCE} || '/root/reference';
    unshift @INC, "$ref/lib";
}
use Sam::Seq;
use Sam::Alignment;
use Fastq::Seq;

{
    no warnings 'redefine';
    *Sam::Seq::alns = sub {
        my ($self, $by_pos) = @_;
        return scalar keys %{ $self->{_alns} } unless wantarray;
        my @a = map { $self->{_alns}{$_} } sort { $a <=> $b } keys %{ $self->{_alns} };
        @a = sort { $a->{pos} <=> $b->{pos} } @a if $by_pos;
        return @a;
    };
}

$SIG{__WARN__} = sub { };   # the reference warns on undef lookups it tolerates

my %DEF = (coverage => 11.25, use_ref_qual => 1, detect_chimera => 0,
           max_ins_length => 0, qual_weighted => 0, noref => 0);

sub run_case {
    my ($name, $par, $ref_lines, $sam_lines) = @_;
    my %p = (%DEF, %$par);

    # bam2cns:227-237 (cfg: sr-trim 1, sr-indel-taboo-length 7, sr-indel-taboo 0.1)
    Sam::Seq->Trim(1);
    Sam::Seq->InDelTabooLength(7);
    Sam::Seq->InDelTaboo(0.1);
    Sam::Seq->MaxCoverage($p{coverage});
    Sam::Seq->BinSize(20);
    Sam::Seq->MaxInsLength($p{max_ins_length});

    my $ref = Fastq::Seq->new(@$ref_lines, phred_offset => 33);
    my $out = ">>CASE $name\n";
    my @kept;
    my $ok = eval {
        my $sso = Sam::Seq->new(
            id  => $ref->id,
            len => length($ref->seq),
            ($p{noref} ? () : (ref => $ref)),
        );
        my @iid;
        for my $l (@$sam_lines) {
            my $aln = Sam::Alignment->new($l);
            die "no seq\n" if $aln->seq eq '*';
            push @iid, $sso->add_aln_by_score($aln);
        }
        @kept = map { (defined $_ && $_ && exists $sso->{_alns}{$_}) ? 1 : 0 } @iid;

        my @mcrs;
        my $desc = $ref->desc;
        if (!$p{noref} && defined $desc) {
            while ($desc =~ /MCR\d+:(\d+),(\d+)/g) { push @mcrs, [ $1, $2 ]; }
        }
        my $con = $sso->consensus(
            use_ref_qual  => ($p{noref} ? 0 : $p{use_ref_qual}),
            ignore_coords => [@mcrs],
            qual_weighted => $p{qual_weighted},
        );
        my $chim = '';
        if ($p{detect_chimera}) {
            my @coords = $sso->chimera();
            my %cg = (M => 0, I => 0, D => 0);
            for my $c (@coords) {
                my ($fr, $to, $sc) = (@{ $c->{col_range} }, $c->{score});
                # same m//g walk as the reference (pos() persists across coords)
                while ($con->{cigar} =~ m/(\d+)(\w)/g && ($cg{M} + $cg{I} < $fr)) {
                    $cg{$2} += $1;
                }
                my $pc = $cg{D} - $cg{I};
                $chim .= sprintf("%s\t%d\t%d\t%s\n", $sso->id, $fr + $pc, $to + $pc, $sc);
            }
        }
        my $fq = "$con";
        chomp $fq;
        $out .= ">>FASTQ\n$fq\n>>TRACE\n" . ($con->{trace} // '') . "\n>>CHIM\n$chim";
        1;
    };
    if (!$ok) { print STDERR "$name: $@" if $ENV{GOLDEN_DEBUG};
        $out = ">>CASE $name\n>>ERROR 1\n";
    }
    $out .= ">>KEPT\n" . join('', @kept) . "\n>>END\n";
    print $out;
}

my ($name, %par, @ref, @sam, $sect);
while (my $line = <>) {
    chomp $line;
    if ($line =~ /^>>CASE (.*)/) { ($name, %par, @ref, @sam, $sect) = ($1); %par = (); @ref = (); @sam = (); $sect = ''; }
    elsif ($line =~ /^>>PARAM (\S+) (.*)/) { $par{$1} = $2; }
    elsif ($line eq '>>REF') { $sect = 'ref'; }
    elsif ($line eq '>>SAM') { $sect = 'sam'; }
    elsif ($line eq '>>END') { run_case($name, \%par, [@ref], [@sam]); }
    elsif ($sect eq 'ref') { push @ref, $line; }
    elsif ($sect eq 'sam') { push @sam, $line if length $line; }
}
